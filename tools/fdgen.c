/* fdgen.c -- seeded synthetic Solana-transaction workloads for the verify
   benchmarks and parity tests.

   Signing uses the system OpenSSL (libcrypto, EVP Ed25519): an independent
   RFC 8032 implementation, so generated signatures cross-check both the CPU
   oracle and the GPU engine.  Neither the oracle nor the engine is used
   here.  Deterministic: transaction i depends only on (seed, i), never on
   the thread count.

   Payload layout (legacy Solana transaction, src/ballet/txn/fd_txn.h):
     [sig_cnt][sig_cnt x 64-B signatures][message]
     message = [sig_cnt][ro_signed=0][ro_unsigned=1][acct_cnt][acct_cnt x 32-B keys]
               [32-B blockhash][instr_cnt=1][prog_idx][n_idx][idx...][data_len][data]
   The first sig_cnt account keys are the signers' public keys. */
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint32_t msg_off, msg_sz, sig_off, pub_off, sig_cnt;
} fdgen_txn_t;

static uint64_t splitmix64(uint64_t *s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static void rng_bytes(uint64_t *s, uint8_t *p, size_t n) {
  while (n) { uint64_t r = splitmix64(s); size_t k = n < 8 ? n : 8; memcpy(p, &r, k); p += k; n -= k; }
}
static uint32_t rng_below(uint64_t *s, uint32_t n) { return (uint32_t)(splitmix64(s) % n); }

static int derive_pub(const uint8_t prv[32], uint8_t pub[32]) {
  EVP_PKEY *pk = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, NULL, prv, 32);
  if (!pk) return -1;
  size_t pl = 32;
  int ok = EVP_PKEY_get_raw_public_key(pk, pub, &pl) == 1 && pl == 32;
  EVP_PKEY_free(pk);
  return ok ? 0 : -1;
}

static int sign_only(const uint8_t prv[32], const uint8_t *msg, size_t msg_sz, uint8_t sig[64]) {
  EVP_PKEY *pk = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, NULL, prv, 32);
  if (!pk) return -1;
  EVP_MD_CTX *ctx = EVP_MD_CTX_new();
  size_t sl = 64;
  int ok = ctx && EVP_DigestSignInit(ctx, NULL, NULL, NULL, pk) == 1 &&
           EVP_DigestSign(ctx, sig, &sl, msg, msg_sz) == 1 && sl == 64;
  EVP_MD_CTX_free(ctx);
  EVP_PKEY_free(pk);
  return ok ? 0 : -1;
}

/* Optional key pool: signers drawn from `cnt` precomputed key pairs
   (recurring signers, as fee payers and vote authorities are in real
   traffic; also halves the signing cost of large parity sets). */
typedef struct {
  uint64_t cnt;
  const uint8_t *prv, *pub;   /* cnt x 32 B each */
} key_pool_t;

/* Build one transaction at p (capacity `stride`).  Returns payload size or 0.
   corrupt_mode 0: a random one of 1-3; 1 signature bit, 2 message bit,
   3 public-key bit, 4 a bit of R (the signature's first 32 bytes). */
static uint32_t build_txn(uint64_t seed, uint64_t idx, int multi, uint32_t msg_lo, uint32_t msg_hi, uint32_t max_sigs,
                          double corrupt_frac, int corrupt_mode, const key_pool_t *pool, uint8_t *p, uint32_t stride,
                          fdgen_txn_t *t, uint64_t base_off, uint8_t *mode_out) {
  uint64_t s = seed ^ (idx * 0xd1342543de82ef95ULL);
  splitmix64(&s);
  const uint32_t n = multi ? 1u + rng_below(&s, max_sigs) : 1u;
  uint32_t extra = multi ? 1u + rng_below(&s, 3) : 2u;            /* non-signer accounts (>= 1: program id) */
  const uint32_t max_msg = multi ? 1232u - 1u - 64u * n : 1u << 20;
  while (4u + 32u * (n + extra) + 33u > max_msg && extra > 1) extra--;
  const uint32_t acct = n + extra;
  /* with one instruction: header(3) acct_cnt(1) keys blockhash instr_cnt prog n_idx idx[acct] data_len(<=2) */
  const uint32_t fixed = 3 + 1 + 32 * acct + 32 + 1 + 1 + 1 + acct + 2;
  const int with_instr = fixed + 4 <= max_msg;
  uint32_t msg_sz;
  if (multi) {
    const uint32_t lo = with_instr ? fixed + 4 : 4 + 32 * acct + 33;
    msg_sz = lo + (with_instr ? rng_below(&s, max_msg - lo + 1) : 0);
  } else {
    msg_sz = msg_lo + rng_below(&s, msg_hi - msg_lo + 1);
    if (msg_sz < fixed + 4) msg_sz = fixed + 4;
  }
  if (1 + 64 * n + msg_sz > stride) return 0;
  uint8_t prv[16][32];
  uint8_t *sigs = p + 1, *msg = p + 1 + 64 * n;
  p[0] = (uint8_t)n;
  uint32_t o = 0;
  msg[o++] = (uint8_t)n; msg[o++] = 0; msg[o++] = 1;
  msg[o++] = (uint8_t)acct;
  for (uint32_t j = 0; j < n; j++) {
    if (pool && pool->cnt) {
      const uint64_t k = splitmix64(&s) % pool->cnt;
      memcpy(prv[j], pool->prv + 32 * k, 32);
      memcpy(msg + o, pool->pub + 32 * k, 32);
    } else {
      rng_bytes(&s, prv[j], 32);
      if (derive_pub(prv[j], msg + o)) return 0;
    }
    o += 32;
  }
  for (uint32_t j = n; j < acct; j++) {
    if (j == acct - 1) memset(msg + o, 0, 32);                       /* system program */
    else rng_bytes(&s, msg + o, 32);
    o += 32;
  }
  rng_bytes(&s, msg + o, 32); o += 32;                               /* recent blockhash */
  if (!with_instr) {
    msg[o++] = 0;                                                    /* instr_cnt = 0 */
    goto sign;
  }
  msg[o++] = 1;                                                      /* instr_cnt */
  msg[o++] = (uint8_t)(acct - 1);                                    /* program id index */
  msg[o++] = (uint8_t)acct;
  for (uint32_t j = 0; j < acct; j++) msg[o++] = (uint8_t)j;
  /* instruction data length as a minimal compact-u16 */
  if (msg_sz - o == 129) msg_sz--;                                    /* 128 needs 2 B, 127 fits 1 B */
  const uint32_t rem = msg_sz - o;
  uint32_t data_len;
  {
  if (rem - 1 < 128) { data_len = rem - 1; msg[o++] = (uint8_t)data_len; }
  else { data_len = rem - 2; msg[o++] = (uint8_t)(0x80 | (data_len & 0x7f)); msg[o++] = (uint8_t)(data_len >> 7); }
  }
  rng_bytes(&s, msg + o, data_len); o += data_len;
sign:
  for (uint32_t j = 0; j < n; j++)
    if (sign_only(prv[j], msg, msg_sz, sigs + 64 * j)) return 0;
  /* corruption: exactly one bit flip in a signature, the message or a public key */
  uint8_t mode = 0;
  if ((double)(splitmix64(&s) >> 11) * (1.0 / 9007199254740992.0) < corrupt_frac) {
    mode = corrupt_mode ? (uint8_t)corrupt_mode : (uint8_t)(1 + rng_below(&s, 3));
    const uint32_t j = rng_below(&s, n);
    if (mode == 1) { uint32_t b = rng_below(&s, 512); sigs[64 * j + b / 8] ^= (uint8_t)(1u << (b & 7)); }
    if (mode == 2) { uint32_t b = rng_below(&s, 8 * msg_sz); msg[b / 8] ^= (uint8_t)(1u << (b & 7)); }
    if (mode == 3) { uint32_t b = rng_below(&s, 256); msg[4 + 32 * j + b / 8] ^= (uint8_t)(1u << (b & 7)); }
    if (mode == 4) { uint32_t b = rng_below(&s, 256); sigs[64 * j + b / 8] ^= (uint8_t)(1u << (b & 7)); }
  }
  const uint32_t payload = 1 + 64 * n + msg_sz;
  t->sig_cnt = n;
  t->sig_off = (uint32_t)(base_off + 1);
  t->msg_off = (uint32_t)(base_off + 1 + 64 * n);
  t->msg_sz = msg_sz;
  t->pub_off = t->msg_off + 4;
  if (mode_out) *mode_out = mode;
  return payload;
}

typedef struct {
  uint64_t n, seed, lo, hi;
  int multi;
  uint32_t msg_lo, msg_hi, max_sigs, stride;
  double corrupt;
  int corrupt_mode;
  const key_pool_t *pool;
  uint8_t *arena;
  fdgen_txn_t *txns;
  uint8_t *modes;
  int err;
} job_t;

static void *worker(void *a) {
  job_t *j = (job_t *)a;
  for (uint64_t i = j->lo; i < j->hi; i++) {
    uint8_t *p = j->arena + i * (uint64_t)j->stride;
    if (!build_txn(j->seed, i, j->multi, j->msg_lo, j->msg_hi, j->max_sigs, j->corrupt, j->corrupt_mode, j->pool, p,
                   j->stride, &j->txns[i], i * (uint64_t)j->stride, j->modes ? &j->modes[i] : NULL)) {
      j->err = 1; return NULL;
    }
  }
  return NULL;
}

typedef struct {
  uint64_t lo, hi, seed;
  uint8_t *prv, *pub;
  int err;
} pool_job_t;

static void *pool_worker(void *a) {
  pool_job_t *j = (pool_job_t *)a;
  for (uint64_t k = j->lo; k < j->hi; k++) {
    uint64_t s = j->seed ^ (k * 0x9e3779b97f4a7c15ULL) ^ 0x6b65795f706f6f6cULL;
    rng_bytes(&s, j->prv + 32 * k, 32);
    if (derive_pub(j->prv + 32 * k, j->pub + 32 * k)) { j->err = 1; return NULL; }
  }
  return NULL;
}

/* Generates n transactions at fixed stride `stride` bytes in `arena`
   (capacity n*stride).  multi=0: one signature, msg_sz ~ U[msg_lo, msg_hi]
   (cfg1); multi=1: sig_cnt ~ U{1..max_sigs}, payload <= 1232 B (cfg3).
   corrupt_frac of the transactions get one bit flipped (modes[i]: 0 none,
   1 signature, 2 message, 3 public key, 4 R; corrupt_mode 0 picks one of
   1-3 at random, else forces it).  key_pool 0: a fresh key pair per signer;
   K > 0: signers drawn from K seeded key pairs.  Returns 0 on success. */
int fdgen_txns_ex(uint64_t n, uint64_t seed, int multi, uint32_t msg_lo, uint32_t msg_hi, uint32_t max_sigs,
                  double corrupt_frac, int corrupt_mode, uint64_t key_pool, uint32_t stride, uint8_t *arena,
                  fdgen_txn_t *txns, uint8_t *modes, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 128) nthreads = 128;
  if (max_sigs < 1 || max_sigs > 16 || (!multi && msg_hi < msg_lo) || corrupt_mode < 0 || corrupt_mode > 4 ||
      key_pool > (1ull << 24))
    return -1;
  key_pool_t pool = {0, NULL, NULL};
  pthread_t th[128];
  if (key_pool) {
    uint8_t *prv = malloc(32 * key_pool), *pub = malloc(32 * key_pool);
    if (!prv || !pub) { free(prv); free(pub); return -3; }
    pool_job_t pj[128];
    int perr = 0;
    for (int t = 0; t < nthreads; t++) {
      pj[t] = (pool_job_t){key_pool * (uint64_t)t / (uint64_t)nthreads, key_pool * (uint64_t)(t + 1) / (uint64_t)nthreads,
                           seed, prv, pub, 0};
      pthread_create(&th[t], NULL, pool_worker, &pj[t]);
    }
    for (int t = 0; t < nthreads; t++) { pthread_join(th[t], NULL); perr |= pj[t].err; }
    if (perr) { free(prv); free(pub); return -2; }
    pool = (key_pool_t){key_pool, prv, pub};
  }
  memset(arena, 0, n * (uint64_t)stride);
  job_t jobs[128];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (job_t){n, seed, n * (uint64_t)t / (uint64_t)nthreads, n * (uint64_t)(t + 1) / (uint64_t)nthreads,
                      multi, msg_lo, msg_hi, max_sigs, stride, corrupt_frac, corrupt_mode, &pool, arena, txns, modes,
                      0};
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  int err = 0;
  for (int t = 0; t < nthreads; t++) { pthread_join(th[t], NULL); err |= jobs[t].err; }
  free((void *)pool.prv); free((void *)pool.pub);
  return err ? -2 : 0;
}

int fdgen_txns(uint64_t n, uint64_t seed, int multi, uint32_t msg_lo, uint32_t msg_hi, uint32_t max_sigs,
               double corrupt_frac, uint32_t stride, uint8_t *arena, fdgen_txn_t *txns, uint8_t *modes,
               int nthreads) {
  return fdgen_txns_ex(n, seed, multi, msg_lo, msg_hi, max_sigs, corrupt_frac, 0, 0, stride, arena, txns, modes,
                       nthreads);
}

/* Plain RFC 8032 keygen + sign of caller-provided messages (test fixtures). */
int fdgen_sign(const uint8_t prv[32], const uint8_t *msg, uint64_t msg_sz, uint8_t pub[32], uint8_t sig[64]) {
  if (derive_pub(prv, pub)) return -1;
  return sign_only(prv, msg, msg_sz, sig);
}
