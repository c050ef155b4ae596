/* fdt_callers.cpp -- the other callers of the verify API, batched over a
   verifier:

     replay   fd_executor_txn_verify (src/flamenco/runtime/fd_executor.c:
              1157-1185) runs fd_ed25519_verify_batch_single_msg on each
              parsed transaction of a block, one at a time;
              fdgpu_replay_verify takes a whole block's raw transactions,
              parses them (fdt_txn_parse) and verifies them in batches;
     shreds   fd_fec_resolver.c:438 checks each new FEC set's merkle root
              with fd_ed25519_verify(root, 32, sig, leader_pubkey);
              fdgpu_fec_roots_verify verifies many roots in one batch
              (32-byte messages, single signatures).

   Both cut the work into batches within the verifier's limits, keep up to
   two batches in flight (the next one is staged while the GPU runs the
   previous) and return one fd_ed25519 code per item. */
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../../include/fd_verify_tile.h"

namespace {

struct Chunk {
  std::vector<uint8_t> arena;
  std::vector<fdgpu_txn_t> txns;
  std::vector<uint64_t> items;     /* caller's index of each txn */
  int64_t ticket = -1;
};

/* Submit / poll with at most two chunks in flight; codes written per item. */
struct Pipe {
  Pipe(fdgpu_verifier_t v_, int8_t *codes_) : v(v_), codes(codes_) {}
  fdgpu_verifier_t v;
  int8_t *codes;
  Chunk slot[2];
  int head = 0, cnt = 0;
  std::vector<int8_t> buf;

  int drain_one() {
    Chunk &c = slot[head];
    buf.resize(std::max<size_t>(c.txns.size(), 1));
    const int r = v.poll(v.ctx, c.ticket, buf.data(), 1);
    if (r != FDGPU_OK) return r < 0 ? r : FDGPU_ERR_DEVICE;
    for (size_t i = 0; i < c.items.size(); i++) codes[c.items[i]] = buf[i];
    head ^= 1;
    cnt--;
    return 0;
  }

  /* the chunk to fill next (drains the oldest when both are busy) */
  int next(Chunk **out) {
    if (cnt == 2) {
      const int r = drain_one();
      if (r) return r;
    }
    Chunk &c = slot[(head + cnt) & 1];
    c.arena.clear(); c.txns.clear(); c.items.clear();
    *out = &c;
    return 0;
  }

  int submit(Chunk &c) {
    if (c.txns.empty()) return 0;
    int64_t tk;
    while ((tk = v.submit(v.ctx, c.arena.data(), c.arena.size(), c.txns.data(), c.txns.size())) == FDGPU_ERR_FULL) {
      if (!cnt) return FDGPU_ERR_FULL;
      const int r = drain_one();
      if (r) return r;
    }
    if (tk < 0) return (int)tk;
    c.ticket = tk;
    cnt++;
    return 0;
  }

  int finish() {
    while (cnt) {
      const int r = drain_one();
      if (r) return r;
    }
    return 0;
  }
};

}  // namespace

extern "C" {

int fdgpu_replay_verify(fdgpu_verifier_t v, const uint8_t *payloads, const uint64_t *off, const uint32_t *sz,
                        uint64_t n, uint64_t batch_txn_max, uint64_t batch_bytes_max, int8_t *codes) {
  if (!v.submit || !v.poll || !codes || (n && (!payloads || !off || !sz)) || !batch_txn_max ||
      batch_bytes_max < FDT_TXN_MTU)
    return FDGPU_ERR_INVAL;
  Pipe p(v, codes);
  alignas(8) uint8_t txn_buf[FDT_TXN_MAX_SZ];
  Chunk *c = nullptr;
  int r = p.next(&c);
  for (uint64_t i = 0; i < n && !r; i++) {
    const uint8_t *raw = payloads + off[i];
    const uint64_t psz = std::min<uint64_t>(sz[i], FDT_TXN_MTU);
    if (!fdt_txn_parse(raw, psz, txn_buf, nullptr)) { codes[i] = FDGPU_REPLAY_PARSE_FAIL; continue; }
    const fdt_txn_t *t = (const fdt_txn_t *)txn_buf;
    if (c->txns.size() == batch_txn_max || c->arena.size() + psz > batch_bytes_max) {
      r = p.submit(*c);
      if (!r) r = p.next(&c);
      if (r) break;
    }
    const uint32_t base = (uint32_t)c->arena.size();
    c->arena.insert(c->arena.end(), raw, raw + psz);
    /* the descriptor fields fd_executor_txn_verify reads (fd_executor.c:1167-1175) */
    fdgpu_txn_t d;
    d.sig_off = base + t->signature_off;
    d.pub_off = base + t->acct_addr_off;
    d.msg_off = base + t->message_off;
    d.msg_sz = (uint32_t)(psz - t->message_off);
    d.sig_cnt = t->signature_cnt;
    c->txns.push_back(d);
    c->items.push_back(i);
  }
  if (!r) r = p.submit(*c);
  if (!r) r = p.finish();
  return r;
}

int fdgpu_fec_roots_verify(fdgpu_verifier_t v, const uint8_t *roots, const uint8_t *sigs, const uint8_t *pubkeys,
                           int shared_pubkey, uint64_t n, uint64_t batch_max, int8_t *codes) {
  if (!v.submit || !v.poll || !codes || (n && (!roots || !sigs || !pubkeys)) || !batch_max)
    return FDGPU_ERR_INVAL;
  Pipe p(v, codes);
  Chunk *c = nullptr;
  int r = p.next(&c);
  for (uint64_t i = 0; i < n && !r; i++) {
    if (c->txns.size() == batch_max) {
      r = p.submit(*c);
      if (!r) r = p.next(&c);
      if (r) break;
    }
    /* item = sig[64] | pub[32] | root[32]: fd_ed25519_verify(root, 32, sig, pub) */
    const uint32_t base = (uint32_t)c->arena.size();
    c->arena.insert(c->arena.end(), sigs + 64 * i, sigs + 64 * i + 64);
    const uint8_t *pk = pubkeys + (shared_pubkey ? 0 : 32 * i);
    c->arena.insert(c->arena.end(), pk, pk + 32);
    c->arena.insert(c->arena.end(), roots + 32 * i, roots + 32 * i + 32);
    fdgpu_txn_t d;
    d.sig_off = base;
    d.pub_off = base + 64;
    d.msg_off = base + 96;
    d.msg_sz = 32;
    d.sig_cnt = 1;
    c->txns.push_back(d);
    c->items.push_back(i);
  }
  if (!r) r = p.submit(*c);
  if (!r) r = p.finish();
  return r;
}

}  // extern "C"
