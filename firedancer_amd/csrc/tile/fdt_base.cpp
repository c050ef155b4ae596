/* fdt_base.cpp -- host-side wire formats around the verify stage:
   tango frag metadata / mcache / compact dcache, tcache, fd_hash and the
   transaction parser (include/fd_verify_tile.h lists the reference lines
   each one restates).  Plain C++17, no GPU code. */
#include <atomic>
#include <cstring>

#include "../../../include/fd_verify_tile.h"
#include "../fdt_hash.h"
#include "../fdt_parse.h"

namespace {

inline uint64_t ld_acq(const uint64_t *p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline void st_rel(uint64_t *p, uint64_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }

}  // namespace

extern "C" {

/* ------------------------------------------------------------ mcache */

uint64_t fdt_frag_meta_ctl(uint64_t orig, int som, int eom, int err) {
  return (uint64_t)(som != 0) | ((uint64_t)(eom != 0) << 1) | ((uint64_t)(err != 0) << 2) | (orig << 3);
}

/* fd_mcache.c:64-69: the line of seq s starts out holding s-1 (so a
   consumer waiting for s sees "not yet") with ctl = som|eom|err. */
void fdt_mcache_init(fdt_frag_meta_t *mcache, uint64_t depth, uint64_t seq0) {
  std::memset(mcache, 0, depth * sizeof(fdt_frag_meta_t));
  for (uint64_t i = 0; i < depth; i++) {
    const uint64_t s = seq0 + i;
    fdt_frag_meta_t &m = mcache[s & (depth - 1)];
    m.seq = s - 1;
    m.ctl = (uint16_t)fdt_frag_meta_ctl(0, 1, 1, 1);
  }
  std::atomic_thread_fence(std::memory_order_release);
}

/* fd_mcache.h:299-322: mark the line as being rewritten (seq-1), write the
   body, then expose seq.  Release ordering makes the body visible before
   the final seq on any consumer that acquires it. */
void fdt_mcache_publish(fdt_frag_meta_t *mcache, uint64_t depth, uint64_t seq, uint64_t sig, uint64_t chunk,
                        uint64_t sz, uint64_t ctl, uint64_t tsorig, uint64_t tspub) {
  fdt_frag_meta_t *m = mcache + (seq & (depth - 1));
  st_rel(&m->seq, seq - 1);
  std::atomic_thread_fence(std::memory_order_release);
  m->sig = sig;
  m->chunk = (uint32_t)chunk;
  m->sz = (uint16_t)sz;
  m->ctl = (uint16_t)ctl;
  m->tsorig = (uint32_t)tsorig;
  m->tspub = (uint32_t)tspub;
  st_rel(&m->seq, seq);
}

/* One poll of FD_MCACHE_WAIT (fd_mcache.h:574-601): read seq, copy the
   line, re-read seq; the copy is trusted only when both reads agree. */
int fdt_mcache_poll(const fdt_frag_meta_t *mcache, uint64_t depth, uint64_t seq, fdt_frag_meta_t *meta,
                    uint64_t *seq_found) {
  const fdt_frag_meta_t *m = mcache + (seq & (depth - 1));
  const uint64_t s0 = ld_acq(&m->seq);
  fdt_frag_meta_t copy;
  std::memcpy(&copy, (const void *)m, sizeof copy);
  std::atomic_thread_fence(std::memory_order_acquire);
  const uint64_t s1 = ld_acq(&m->seq);
  if (seq_found) *seq_found = s0;
  const int64_t diff = (int64_t)(s0 - seq);
  if (s0 != s1 || diff < 0) return 0;    /* being written, or not yet published */
  if (diff > 0) return -1;               /* overrun */
  copy.seq = s0;
  std::memcpy((void *)meta, &copy, sizeof copy);   /* caller storage need not be 32-B aligned */
  return 1;
}

uint64_t fdt_mcache_query(const fdt_frag_meta_t *mcache, uint64_t depth, uint64_t seq) {
  return ld_acq(&mcache[seq & (depth - 1)].seq);
}

/* ------------------------------------------------------------ dcache */

/* fd_dcache.h:214: chunks for a worst-case frag, rounded to a chunk pair */
uint64_t fdt_dcache_chunk_mtu(uint64_t mtu) { return ((mtu + 2 * FDT_CHUNK_SZ - 1) >> (1 + FDT_CHUNK_LG_SZ)) << 1; }

/* room for chunk_mtu*(depth+2)-1 chunks (fd_dcache.h:220-260), rounded up */
uint64_t fdt_dcache_data_sz(uint64_t mtu, uint64_t depth) {
  return fdt_dcache_chunk_mtu(mtu) * (depth + 2) * FDT_CHUNK_SZ;
}

uint64_t fdt_dcache_wmark(uint64_t chunk0, uint64_t chunk1, uint64_t mtu) {
  (void)chunk0;
  return chunk1 - fdt_dcache_chunk_mtu(mtu);
}

/* fd_dcache.h:262-269 */
uint64_t fdt_dcache_compact_next(uint64_t chunk, uint64_t sz, uint64_t chunk0, uint64_t wmark) {
  chunk += ((sz + 2 * FDT_CHUNK_SZ - 1) >> (1 + FDT_CHUNK_LG_SZ)) << 1;
  return chunk > wmark ? chunk0 : chunk;
}

/* ------------------------------------------------------------ tcache */

namespace {
constexpr uint64_t TCACHE_MAGIC = 0xf17eda2c377ca540ULL;   /* fd_tcache.h:63 */
struct tcache_view {
  uint64_t *hdr;
  uint64_t depth() const { return hdr[1]; }
  uint64_t map_cnt() const { return hdr[2]; }
  uint64_t &oldest() const { return hdr[3]; }
  uint64_t *ring() const { return hdr + 4; }
  uint64_t *map() const { return hdr + 4 + hdr[1]; }
};
inline int msb64(uint64_t x) { return 63 - __builtin_clzll(x); }

/* linear probe from tag & (map_cnt-1) to the tag or the first null slot
   (FD_TCACHE_QUERY, fd_tcache.h:281-295) */
inline bool map_find(const uint64_t *map, uint64_t map_cnt, uint64_t tag, uint64_t &slot) {
  slot = tag & (map_cnt - 1);
  for (;;) {
    const uint64_t t = map[slot];
    if (t == tag) return true;
    if (t == FDT_TCACHE_TAG_NULL) return false;
    slot = (slot + 1) & (map_cnt - 1);
  }
}

/* backward-shift deletion of tag (fd_tcache_remove, fd_tcache.h:306-342):
   after emptying a slot, walk the probe run and pull back every entry
   whose home slot is not cyclically within (hole, slot]. */
void map_remove(uint64_t *map, uint64_t map_cnt, uint64_t tag) {
  if (tag == FDT_TCACHE_TAG_NULL) return;
  uint64_t slot;
  if (!map_find(map, map_cnt, tag, slot)) return;
  const uint64_t mask = map_cnt - 1;
  for (;;) {
    map[slot] = FDT_TCACHE_TAG_NULL;
    const uint64_t hole = slot;
    uint64_t t;
    for (;;) {
      slot = (slot + 1) & mask;
      t = map[slot];
      if (t == FDT_TCACHE_TAG_NULL) return;
      const uint64_t home = t & mask;
      /* stays iff home lies cyclically in (hole, slot] */
      const bool stays = (hole < slot) ? (hole < home && home <= slot) : (hole < home || home <= slot);
      if (!stays) break;
    }
    map[hole] = t;
  }
}
}  // namespace

uint64_t fdt_tcache_map_cnt_default(uint64_t depth) {
  if (!depth || depth == UINT64_MAX) return 0;
  const int lg = msb64(depth + 1) + 2;                    /* FD_TCACHE_SPARSE_DEFAULT = 2 */
  if (lg > 63) return 0;
  return 1ULL << lg;
}

uint64_t fdt_tcache_footprint(uint64_t depth, uint64_t map_cnt) {
  if (!map_cnt) map_cnt = fdt_tcache_map_cnt_default(depth);
  if (!depth || !map_cnt || (map_cnt & (map_cnt - 1)) || map_cnt < depth + 2) return 0;
  uint64_t words = 4 + depth;                              /* overflow guards as fd_tcache.c:15-19 */
  if (words < depth) return 0;
  words += map_cnt;
  if (words < map_cnt || words > UINT64_MAX / 8) return 0;
  const uint64_t bytes = words * 8, fp = (bytes + 127) & ~127ULL;
  return fp < bytes ? 0 : fp;
}

void *fdt_tcache_new(void *mem, uint64_t depth, uint64_t map_cnt) {
  if (!map_cnt) map_cnt = fdt_tcache_map_cnt_default(depth);
  if (!mem || !fdt_tcache_footprint(depth, map_cnt)) return nullptr;
  uint64_t *h = (uint64_t *)mem;
  h[0] = TCACHE_MAGIC; h[1] = depth; h[2] = map_cnt; h[3] = 0;
  fdt_tcache_reset(mem);
  return mem;
}

void fdt_tcache_reset(void *tc) {
  tcache_view v{(uint64_t *)tc};
  std::memset(v.ring(), 0, v.depth() * 8);
  std::memset(v.map(), 0, v.map_cnt() * 8);
  v.oldest() = 0;
}

int fdt_tcache_query(const void *tc, uint64_t tag) {
  tcache_view v{(uint64_t *)tc};
  uint64_t slot;
  return map_find(v.map(), v.map_cnt(), tag, slot) ? 1 : 0;
}

/* FD_TCACHE_INSERT (fd_tcache.h:373-404): not LRU -- a duplicate leaves
   the cache untouched; a new tag takes the oldest ring slot and the
   evicted tag leaves the map. */
int fdt_tcache_insert(void *tc, uint64_t tag) {
  tcache_view v{(uint64_t *)tc};
  uint64_t slot;
  if (map_find(v.map(), v.map_cnt(), tag, slot)) return 1;
  v.map()[slot] = tag;
  uint64_t &old = v.oldest();
  const uint64_t evict = v.ring()[old];
  v.ring()[old] = tag;
  old = (old + 1 >= v.depth()) ? 0 : old + 1;
  map_remove(v.map(), v.map_cnt(), evict);
  return 0;
}

void fdt_tcache_prefetch(const void *tc, uint64_t tag) {
  tcache_view v{(uint64_t *)const_cast<void *>(tc)};
  __builtin_prefetch(v.map() + (tag & (v.map_cnt() - 1)));
}

void fdt_tcache_prefetch_evict(const void *tc, uint64_t ahead) {
  tcache_view v{(uint64_t *)const_cast<void *>(tc)};
  uint64_t k = v.oldest() + ahead;
  while (k >= v.depth()) k -= v.depth();
  const uint64_t victim = v.ring()[k];
  if (victim != FDT_TCACHE_TAG_NULL) __builtin_prefetch(v.map() + (victim & (v.map_cnt() - 1)));
}

uint64_t fdt_tcache_insert_many(void *tc, const uint64_t *tags, uint64_t n) {
  uint64_t dup = 0;
  for (uint64_t i = 0; i < n; i++) dup += (uint64_t)fdt_tcache_insert(tc, tags[i]);
  return dup;
}

void fdt_tagring_init(fdt_tagring_t *r, uint64_t depth) {
  std::memset(r, 0, sizeof *r);
  r->depth = depth < 1 ? 1 : depth > FDT_TAGRING_MAX ? FDT_TAGRING_MAX : depth;
}

int fdt_tagring_query(const fdt_tagring_t *r, uint64_t tag) {
  if (tag == FDT_TCACHE_TAG_NULL) return 1;
  uint64_t hit = 0;
  for (uint64_t i = 0; i < r->depth; i++) hit |= (uint64_t)(r->tag[i] == tag);   /* no early exit: vectorised */
  return hit ? 1 : 0;
}

int fdt_tagring_insert(fdt_tagring_t *r, uint64_t tag) {
  if (fdt_tagring_query(r, tag)) return 1;
  r->tag[r->oldest] = tag;                       /* the evicted (oldest) tag leaves with its slot */
  r->oldest = r->oldest + 1 >= r->depth ? 0 : r->oldest + 1;
  return 0;
}

/* -------------------------------------------------------------- hash */

/* xxhash-r39 over 64-bit lanes (fd_hash.c:12-73): ../fdt_hash.h, shared
   with the GPU's frag finish kernel. */
uint64_t fdt_hash(uint64_t seed, const void *buf, uint64_t sz) {
  const uint8_t *p = (const uint8_t *)buf;
  if (sz == 64) {                               /* the dedup tag: 8-byte loads, the compiler's own */
    uint64_t w[8];
    std::memcpy(w, p, 64);
    uint64_t a = seed + FDT_HASH_P1 + FDT_HASH_P2, b = seed + FDT_HASH_P2, c = seed, d = seed - FDT_HASH_P1;
    for (int i = 0; i < 8; i += 4) {
      a = fdt_hash_round(a, w[i]); b = fdt_hash_round(b, w[i + 1]);
      c = fdt_hash_round(c, w[i + 2]); d = fdt_hash_round(d, w[i + 3]);
    }
    uint64_t h = fdt_hash_rotl(a, 1) + fdt_hash_rotl(b, 7) + fdt_hash_rotl(c, 12) + fdt_hash_rotl(d, 18);
    h = fdt_hash_merge(h, a); h = fdt_hash_merge(h, b); h = fdt_hash_merge(h, c); h = fdt_hash_merge(h, d);
    h += 64;
    h ^= h >> 33; h *= FDT_HASH_P2; h ^= h >> 29; h *= FDT_HASH_P3; h ^= h >> 32;
    return h;
  }
  return fdt_hash_core(seed, p, sz);
}

/* --------------------------------------------------------------- txn */

uint64_t fdt_txn_footprint(uint64_t instr_cnt, uint64_t lut_cnt) {
  return sizeof(fdt_txn_t) + instr_cnt * sizeof(fdt_txn_instr_t) + lut_cnt * sizeof(fdt_txn_acct_addr_lut_t);
}

}  // extern "C"

static_assert(sizeof(fdt_frag_meta_t) == 32, "fd_frag_meta_t is 32 B");
static_assert(sizeof(fdt_txn_t) == 20, "fd_txn_t header is 20 B");
static_assert(sizeof(fdt_txn_instr_t) == 10, "fd_txn_instr_t is 10 B");
static_assert(sizeof(fdt_txn_acct_addr_lut_t) == 8, "fd_txn_acct_addr_lut_t is 8 B");

/* fd_txn_parse (fd_txn_parse.c:7-243): the parser lives in
   ../fdt_parse.h, shared with the GPU ingest kernel; this wrapper keeps the
   reference's counters (a success count and a ring of failure reasons). */
extern "C" uint64_t fdt_txn_parse(const uint8_t *payload, uint64_t payload_sz, void *out_buf,
                                  fdt_txn_parse_counters_t *counters) {
  uint64_t why = 0;
  const uint64_t fp = fdt_parse_core(payload, payload_sz, (fdt_txn_t *)out_buf, &why);
  if (counters) {
    if (fp) counters->success_cnt++;
    else counters->failure_ring[counters->failure_cnt++ % 32] = why;
  }
  return fp;
}

/* fdt_peek_core (../fdt_parse.h): the footprint a successful parse would
   have, from the payload's counts */
extern "C" uint64_t fdt_txn_peek(const uint8_t *payload, uint64_t payload_sz, uint64_t *sig_cnt) {
  return fdt_peek_core(payload, payload_sz, sig_cnt);
}
