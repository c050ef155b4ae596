/* fdt_vtile.cpp -- the verify tile around the GPU engine, the multi-GPU
   dispatcher, the dedup tile and a line-rate frag producer
   (include/fd_verify_tile.h).

   Verify tile (src/app/fdctl/run/tiles/fd_verify.c:36-148 and
   fd_verify.h:45-89 restated for batched, asynchronous verification):

     ingest   FD_MCACHE_WAIT-style polls of the in mcache; a frag outside
              this tile's round-robin share is skipped (fd_verify.c:46); the
              payload is copied into the open batch, the line re-checked for
              overrun (fd_mux.c:641-647), then fd_txn_parse'd into the
              batch's trailer area; parse failures are filtered
              (fd_verify.c:117-121).
     verify   the batch's per-transaction descriptors {msg, sigs, pubkeys,
              sig_cnt} (fd_verify.h:53-61) go to the verifier as one
              fd_ed25519_verify_batch_single_msg job per txn; up to
              inflight_max batches are outstanding at once.
     resolve  strictly in ingest order, one txn at a time: tag =
              fd_hash(seed, sig0, 64); tcache hit -> DEDUP; verify code != 0
              -> FAILED; else tcache insert and publish
              [payload][pad][fd_txn_t][u16 payload_sz] with sig = tag
              (fd_verify.c:93-147).  Because every earlier txn is resolved
              first, the tcache sees exactly the insert sequence of the
              reference's one-frag-at-a-time loop, so each txn's outcome is
              identical; duplicates are still sent to the GPU (harmless
              extra work) since whether they are duplicates is only known at
              resolution.
   Out-link flow control: with out_fseq set, publishing stops while the
   consumer is a full mcache depth behind (the mux credit check,
   fd_mux.c:548). */
#include <sys/mman.h>
#include <time.h>

#include <algorithm>
#include <cstddef>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <new>
#include <thread>
#include <vector>

#include "../../../include/fd_verify_tile.h"

namespace {

inline uint64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

inline uint64_t align2(uint64_t x) { return (x + 1) & ~1ull; }

/* cycle counter (fd_tickcount) */
inline uint64_t tick() {
#if defined(__x86_64__)
  return __builtin_ia32_rdtsc();
#else
  return now_ns();
#endif
}

}  // namespace

/* ----------------------------------------------------------- dispatch */

struct fdgpu_dispatch {
  std::vector<fdgpu_engine_t *> eng;
  uint32_t next = 0;
  int staged = -1;          /* engine holding the staged slot */
};

namespace {

/* ticket = engine_ticket * n + engine index */
int64_t dispatch_submit(void *ctx, const uint8_t *arena, uint64_t arena_sz, const fdgpu_txn_t *txns, uint64_t n_txn) {
  auto *d = (fdgpu_dispatch *)ctx;
  const uint32_t n = (uint32_t)d->eng.size();
  for (uint32_t k = 0; k < n; k++) {
    const uint32_t idx = (d->next + k) % n;
    const int64_t t = fdgpu_submit(d->eng[idx], arena, arena_sz, txns, n_txn);
    if (t == FDGPU_ERR_FULL) continue;
    if (t < 0) return t;
    d->next = (idx + 1) % n;
    return t * n + idx;
  }
  return FDGPU_ERR_FULL;
}

int dispatch_poll(void *ctx, int64_t ticket, int8_t *codes, int blocking) {
  auto *d = (fdgpu_dispatch *)ctx;
  const int64_t n = (int64_t)d->eng.size();
  if (ticket < 0) return FDGPU_ERR_TICKET;
  return fdgpu_poll(d->eng[ticket % n], ticket / n, codes, blocking);
}

uint8_t *dispatch_stage(void *ctx, uint64_t *cap) {
  auto *d = (fdgpu_dispatch *)ctx;
  if (d->staged >= 0) return nullptr;
  const uint32_t n = (uint32_t)d->eng.size();
  for (uint32_t k = 0; k < n; k++) {
    const uint32_t idx = (d->next + k) % n;
    uint8_t *p = fdgpu_stage_acquire(d->eng[idx], cap);
    if (p) { d->staged = (int)idx; d->next = (idx + 1) % n; return p; }
  }
  return nullptr;
}

int64_t dispatch_submit_staged(void *ctx, uint64_t arena_sz, const fdgpu_txn_t *txns, uint64_t n_txn) {
  auto *d = (fdgpu_dispatch *)ctx;
  if (d->staged < 0) return FDGPU_ERR_INVAL;
  const int idx = d->staged;
  const int64_t t = fdgpu_stage_submit(d->eng[idx], arena_sz, txns, n_txn);
  if (t < 0) return t;
  d->staged = -1;
  return t * (int64_t)d->eng.size() + idx;
}

int dispatch_poll_keep(void *ctx, int64_t ticket, int8_t *codes, int blocking) {
  auto *d = (fdgpu_dispatch *)ctx;
  const int64_t n = (int64_t)d->eng.size();
  if (ticket < 0) return FDGPU_ERR_TICKET;
  return fdgpu_poll_keep(d->eng[ticket % n], ticket / n, codes, blocking);
}

int dispatch_release(void *ctx, int64_t ticket) {
  auto *d = (fdgpu_dispatch *)ctx;
  const int64_t n = (int64_t)d->eng.size();
  if (ticket < 0) return FDGPU_ERR_TICKET;
  return fdgpu_release(d->eng[ticket % n], ticket / n);
}

int64_t dispatch_submit_frags(void *ctx, const uint8_t *arena, uint64_t arena_sz, const fdgpu_frag_ex_t *fx,
                              uint64_t n, uint64_t trailer_sz) {
  auto *d = (fdgpu_dispatch *)ctx;
  const uint32_t ne = (uint32_t)d->eng.size();
  for (uint32_t k = 0; k < ne; k++) {
    const uint32_t idx = (d->next + k) % ne;
    const int64_t t = fdgpu_submit_frags(d->eng[idx], arena, arena_sz, fx, n, trailer_sz);
    if (t == FDGPU_ERR_FULL) continue;
    if (t < 0) return t;
    d->next = (idx + 1) % ne;
    return t * ne + idx;
  }
  return FDGPU_ERR_FULL;
}

int dispatch_poll_frags(void *ctx, int64_t ticket, int8_t *codes, uint8_t *trailers, int blocking) {
  auto *d = (fdgpu_dispatch *)ctx;
  const int64_t n = (int64_t)d->eng.size();
  if (ticket < 0) return FDGPU_ERR_TICKET;
  return fdgpu_poll_frags(d->eng[ticket % n], ticket / n, codes, trailers, blocking);
}

int64_t dispatch_submit_io(void *ctx, const fdgpu_frag_io_t *fio, uint64_t n, uint8_t *out, uint64_t out_sz,
                           uint64_t seed, const fdgpu_link_t *links, uint64_t link_cnt) {
  auto *d = (fdgpu_dispatch *)ctx;
  const uint32_t ne = (uint32_t)d->eng.size();
  for (uint32_t k = 0; k < ne; k++) {
    const uint32_t idx = (d->next + k) % ne;
    const int64_t t = fdgpu_submit_frags_io(d->eng[idx], fio, n, out, out_sz, seed, links, link_cnt);
    if (t == FDGPU_ERR_FULL) continue;
    if (t < 0) return t;
    d->next = (idx + 1) % ne;
    return t * ne + idx;
  }
  return FDGPU_ERR_FULL;
}

int dispatch_poll_io(void *ctx, int64_t ticket, int8_t *codes, uint64_t *tags, uint16_t *out_szs, int blocking) {
  auto *d = (fdgpu_dispatch *)ctx;
  const int64_t n = (int64_t)d->eng.size();
  if (ticket < 0) return FDGPU_ERR_TICKET;
  return fdgpu_poll_frags_io(d->eng[ticket % n], ticket / n, codes, tags, out_szs, blocking);
}

int dispatch_stage_cancel(void *ctx) {
  auto *d = (fdgpu_dispatch *)ctx;
  if (d->staged < 0) return FDGPU_ERR_INVAL;
  const int rc = fdgpu_stage_cancel(d->eng[d->staged]);
  d->staged = -1;
  return rc;
}

}  // namespace

extern "C" {

fdgpu_dispatch_t *fdgpu_dispatch_new(fdgpu_engine_t *const *engines, uint32_t engine_cnt) {
  if (!engines || !engine_cnt) return nullptr;
  auto *d = new (std::nothrow) fdgpu_dispatch;
  if (!d) return nullptr;
  d->eng.assign(engines, engines + engine_cnt);
  for (auto *e : d->eng) if (!e) { delete d; return nullptr; }
  return d;
}

void fdgpu_dispatch_delete(fdgpu_dispatch_t *d) { delete d; }

fdgpu_verifier_t fdgpu_dispatch_verifier(fdgpu_dispatch_t *d) {
  fdgpu_verifier_t v{};
  v.ctx = d;
  v.submit = dispatch_submit;
  v.poll = dispatch_poll;
  v.stage = dispatch_stage;
  v.submit_staged = dispatch_submit_staged;
  v.poll_keep = dispatch_poll_keep;
  v.release = dispatch_release;
  v.stage_cancel = dispatch_stage_cancel;
  v.submit_frags = dispatch_submit_frags;
  v.poll_frags = dispatch_poll_frags;
  v.submit_io = dispatch_submit_io;
  v.poll_io = dispatch_poll_io;
  return v;
}

}  // extern "C"

/* -------------------------------------------------------- verify tile */

namespace {

struct Item {
  uint64_t seq;
  uint32_t pay_off;     /* payload offset in the batch arena */
  uint16_t pay_sz;
  uint16_t txn_sz;      /* parsed fd_txn_t footprint */
  uint32_t txn_off;     /* in the batch trailer area */
  uint32_t tsorig;
};

struct Batch {
  std::vector<uint8_t> arena;       /* payload copies, back to back (when not staged) */
  uint8_t *ap = nullptr;            /* the arena in use: arena.data() or a staged pinned slot */
  uint64_t cap = 0;                 /* its capacity */
  bool staged = false;
  std::vector<uint8_t> trailer;     /* parsed fd_txn_t of each item */
  std::vector<fdgpu_txn_t> txns;    /* one per item */
  std::vector<Item> items;
  std::vector<int8_t> codes;
  uint64_t arena_used = 0, trailer_used = 0;
  uint64_t sig_cnt = 0;             /* signatures the verifier will check (sig_cnt in [1,16] per txn) */
  int64_t ticket = -1;
  bool done = false;
  size_t next = 0;                  /* next item to resolve */
  uint64_t t_first = 0;

  void reset() {
    arena_used = trailer_used = 0;
    sig_cnt = 0;
    txns.clear(); items.clear();
    ticket = -1; done = false; next = 0; t_first = 0;
    ap = nullptr; cap = 0; staged = false;
  }
};

}  // namespace

struct fdgpu_vtile {
  fdgpu_vtile_cfg_t cfg{};
  fdgpu_verifier_t ver{};
  std::vector<uint64_t> tcache_mem;
  void *tcache = nullptr;
  uint64_t rx_seq = 0, out_seq = 0, out_chunk = 0;
  std::vector<Batch *> pool;         /* free batches */
  std::deque<Batch *> inflight;      /* submitted, resolved in order */
  Batch *open = nullptr;             /* being filled */
  std::vector<Batch> storage;
  fdgpu_vtile_stats_t st{};
  std::vector<uint64_t> lat;
  uint64_t log_max = 0;
  std::vector<uint64_t> log_seq;
  std::vector<int8_t> log_code;

  void log(uint64_t seq, int code) {
    if (log_seq.size() < log_max) { log_seq.push_back(seq); log_code.push_back((int8_t)code); }
  }

  int64_t credits() const {
    if (!cfg.out_fseq) return INT64_MAX;
    const uint64_t fseq = __atomic_load_n(cfg.out_fseq, __ATOMIC_ACQUIRE);
    return (int64_t)cfg.out_depth - (int64_t)(out_seq - fseq);
  }

  /* publish one verified txn downstream (fd_verify.c:93-147) */
  void publish(const Batch &b, const Item &it, uint64_t tag) {
    uint8_t *dst = cfg.out_base + (out_chunk << FDT_CHUNK_LG_SZ);
    std::memcpy(dst, b.ap + it.pay_off, it.pay_sz);
    const uint64_t toff = align2(it.pay_sz);
    if (toff != it.pay_sz) dst[it.pay_sz] = 0;
    std::memcpy(dst + toff, b.trailer.data() + it.txn_off, it.txn_sz);
    const uint16_t psz = it.pay_sz;
    std::memcpy(dst + toff + it.txn_sz, &psz, 2);
    const uint64_t new_sz = toff + it.txn_sz + 2;
    fdt_mcache_publish(cfg.out_mcache, cfg.out_depth, out_seq, tag, out_chunk, new_sz, 0, it.tsorig,
                       (uint32_t)now_ns());
    out_seq++;
    out_chunk = fdt_dcache_compact_next(out_chunk, new_sz, cfg.out_chunk0, cfg.out_wmark);
    st.published++;
  }

  /* resolve completed batches in order; returns txns resolved, < 0 on error */
  int64_t resolve() {
    int64_t n = 0;
    while (!inflight.empty()) {
      Batch *b = inflight.front();
      if (!b->done) {
        const uint64_t t0 = now_ns();
        const int rc = b->staged ? ver.poll_keep(ver.ctx, b->ticket, b->codes.data(), 0)
                                 : ver.poll(ver.ctx, b->ticket, b->codes.data(), 0);
        st.poll_ns += now_ns() - t0;
        if (rc == FDGPU_PENDING) break;
        if (rc != FDGPU_OK) return rc;
        b->done = true;
      }
      while (b->next < b->items.size()) {
        if (credits() <= 0) { st.backpressure++; return n; }
        const Item &it = b->items[b->next];
        const uint64_t tag = fdt_hash(cfg.hashmap_seed, b->ap + it.pay_off +
                                      ((const fdt_txn_t *)(b->trailer.data() + it.txn_off))->signature_off, 64);
        int outcome;
        if (fdt_tcache_query(tcache, tag)) outcome = FD_TXN_VERIFY_DEDUP;
        else if (b->codes[b->next] != FD_ED25519_SUCCESS) outcome = FD_TXN_VERIFY_FAILED;
        else outcome = fdt_tcache_insert(tcache, tag) ? FD_TXN_VERIFY_DEDUP : FD_TXN_VERIFY_SUCCESS;
        if (outcome == FD_TXN_VERIFY_SUCCESS) publish(*b, it, tag);
        else if (outcome == FD_TXN_VERIFY_DEDUP) st.dedup++;
        else st.verify_failed++;
        log(it.seq, outcome);
        b->next++;
        n++;
      }
      if (lat.size() < (1u << 22) && !b->items.empty()) lat.push_back(now_ns() - b->t_first);
      if (b->staged) ver.release(ver.ctx, b->ticket);
      inflight.pop_front();
      b->reset();
      pool.push_back(b);
    }
    return n;
  }

  /* ingest available frags into the open batch (stops when it is full) */
  void ingest() {
    const uint64_t t_in = now_ns();
    struct Acc { uint64_t &ns; uint64_t t; ~Acc() { ns += now_ns() - t; } } acc{st.ingest_ns, t_in};
    if (!open) {
      if (pool.empty()) { st.no_slot_steps++; return; }
      Batch *nb = pool.back();
      if (ver.stage) {                                  /* zero-copy: frags go straight to pinned memory */
        uint64_t cap = 0;
        const uint64_t t0 = now_ns();
        uint8_t *p = ver.stage(ver.ctx, &cap);
        const uint64_t dt = now_ns() - t0;
        st.submit_ns += dt;
        acc.t += dt;                                    /* counted as submit time, not ingest */
        if (!p) { st.no_slot_steps++; return; }         /* every slot busy: resolve first */
        nb->ap = p; nb->cap = cap; nb->staged = true;
      } else {
        nb->ap = nb->arena.data(); nb->cap = nb->arena.size();
      }
      pool.pop_back();
      open = nb;
    }
    Batch &b = *open;
    /* room for one more frag: payload bytes, and signatures (a txn sends at
       most 16 to the verifier; more make batch_single_msg fail unverified) */
    while (b.items.size() < cfg.batch_txn_max && b.arena_used + FDT_TPU_MTU <= b.cap &&
           b.sig_cnt + 16 <= cfg.batch_sig_max) {
      fdt_frag_meta_t m;
      uint64_t found;
      const int rc = fdt_mcache_poll(cfg.in_mcache, cfg.in_depth, rx_seq, &m, &found);
      if (rc == 0) break;
      if (rc < 0) {                                     /* overrun: skip to the producer */
        for (uint64_t s = rx_seq; s != found; s++) log(s, FDGPU_VTILE_LOG_LOST);
        st.overrun += found - rx_seq;
        rx_seq = found;
        continue;
      }
      const uint64_t seq = rx_seq++;
      st.in_frags++;
      if (cfg.round_robin_cnt > 1 && seq % cfg.round_robin_cnt != cfg.round_robin_idx) {
        st.filtered_rr++; log(seq, FDGPU_VTILE_LOG_FILTERED); continue;
      }
      if (m.chunk < cfg.in_chunk0 || m.chunk > cfg.in_wmark || m.sz > FDT_TPU_MTU) {
        st.corrupt++; log(seq, FDGPU_VTILE_LOG_LOST); continue;
      }
      uint8_t *pay = b.ap + b.arena_used;
      std::memcpy(pay, cfg.in_base + ((uint64_t)m.chunk << FDT_CHUNK_LG_SZ), m.sz);
      if (fdt_mcache_query(cfg.in_mcache, cfg.in_depth, seq) != seq) {   /* overwritten while copying */
        st.overrun++; log(seq, FDGPU_VTILE_LOG_LOST); continue;
      }
      uint8_t *txn = b.trailer.data() + b.trailer_used;
      const uint64_t tsz = fdt_txn_parse(pay, m.sz, txn, nullptr);
      if (!tsz) { st.parse_fail++; log(seq, FDGPU_VTILE_LOG_PARSE_FAIL); continue; }
      const fdt_txn_t *t = (const fdt_txn_t *)txn;
      fdgpu_txn_t d;
      d.sig_off = (uint32_t)(b.arena_used + t->signature_off);
      d.pub_off = (uint32_t)(b.arena_used + t->acct_addr_off);
      d.msg_off = (uint32_t)(b.arena_used + t->message_off);
      d.msg_sz = (uint32_t)(m.sz - t->message_off);
      d.sig_cnt = t->signature_cnt;
      if (b.items.empty()) b.t_first = now_ns();
      b.items.push_back(Item{seq, (uint32_t)b.arena_used, m.sz, (uint16_t)tsz, (uint32_t)b.trailer_used, m.tsorig});
      b.txns.push_back(d);
      b.arena_used += m.sz;
      b.trailer_used += (tsz + 7) & ~7ull;
      if (t->signature_cnt <= 16) { b.sig_cnt += t->signature_cnt; st.sigs += t->signature_cnt; }
    }
  }

  /* The verifier refused the batch as malformed (e.g. more signatures than
     the engine was opened for): its transactions are failed -- logged as
     FAILED and counted in verify_errors, nothing published -- and the batch
     returns to the pool, so the tile keeps running.  Device errors stay
     fatal (returned from step). */
  void reject_open() {
    Batch *b = open;
    for (const Item &it : b->items) { st.verify_errors++; log(it.seq, FD_TXN_VERIFY_FAILED); }
    if (b->staged && ver.stage_cancel) ver.stage_cancel(ver.ctx);
    b->reset();
    pool.push_back(b);
    open = nullptr;
  }

  /* submit the open batch when full or when its first frag has waited long enough */
  int submit(bool force) {
    if (!open || open->items.empty()) return 0;
    const bool full = open->items.size() >= cfg.batch_txn_max || open->arena_used + FDT_TPU_MTU > open->cap ||
                      open->sig_cnt + 16 > cfg.batch_sig_max;
    if (!full && !force && now_ns() - open->t_first < cfg.batch_wait_ns) return 0;
    if (inflight.size() >= cfg.inflight_max) return 0;
    const uint64_t t0 = now_ns();
    const int64_t t = open->staged
        ? ver.submit_staged(ver.ctx, open->arena_used, open->txns.data(), open->txns.size())
        : ver.submit(ver.ctx, open->ap, open->arena_used, open->txns.data(), open->txns.size());
    st.submit_ns += now_ns() - t0;
    if (t == FDGPU_ERR_FULL) return 0;
    if (t == FDGPU_ERR_INVAL) { reject_open(); return 0; }
    if (t < 0) return (int)t;
    open->ticket = t;
    inflight.push_back(open);
    open = nullptr;
    st.batches++;
    return 1;
  }
};

extern "C" {

fdgpu_vtile_t *fdgpu_vtile_new(const fdgpu_vtile_cfg_t *cfg, fdgpu_verifier_t ver) {
  if (!cfg || !ver.submit || !ver.poll || !cfg->in_mcache || !cfg->out_mcache || !cfg->in_base || !cfg->out_base)
    return nullptr;
  if (ver.stage && (!ver.submit_staged || !ver.poll_keep || !ver.release)) return nullptr;
  if (!cfg->in_depth || (cfg->in_depth & (cfg->in_depth - 1)) || !cfg->out_depth ||
      (cfg->out_depth & (cfg->out_depth - 1)) || !cfg->batch_txn_max || cfg->out_wmark < cfg->out_chunk0)
    return nullptr;
  auto *t = new (std::nothrow) fdgpu_vtile;
  if (!t) return nullptr;
  t->cfg = *cfg;
  t->st.lap_margin_min = UINT64_MAX;                    /* the gather tile's measure; none here */
  if (!t->cfg.round_robin_cnt) t->cfg.round_robin_cnt = 1;
  if (!t->cfg.inflight_max) t->cfg.inflight_max = 2;
  if (!t->cfg.tcache_depth) t->cfg.tcache_depth = FDT_VERIFY_TCACHE_DEPTH;
  /* default: the engine's default max_sig (12 per txn), at least one txn's 16 */
  if (!t->cfg.batch_sig_max) t->cfg.batch_sig_max = std::max<uint64_t>(16, (uint64_t)t->cfg.batch_txn_max * 12);
  if (t->cfg.batch_sig_max < 16) { delete t; return nullptr; }
  if (!cfg->tcache_depth && !t->cfg.tcache_map_cnt) t->cfg.tcache_map_cnt = FDT_VERIFY_TCACHE_MAP_CNT;
  const uint64_t fp = fdt_tcache_footprint(t->cfg.tcache_depth, t->cfg.tcache_map_cnt);
  if (!fp) { delete t; return nullptr; }
  t->tcache_mem.assign(fp / 8, 0);
  t->tcache = fdt_tcache_new(t->tcache_mem.data(), t->cfg.tcache_depth, t->cfg.tcache_map_cnt);
  t->ver = ver;
  t->rx_seq = cfg->in_seq0;
  t->out_seq = cfg->out_seq0;
  t->out_chunk = cfg->out_chunk0;
  const uint32_t nb = t->cfg.inflight_max + 1;
  t->storage.resize(nb);
  for (auto &b : t->storage) {
    b.arena.resize((size_t)t->cfg.batch_txn_max * FDT_TPU_MTU + 256);
    b.trailer.resize((size_t)t->cfg.batch_txn_max * (FDT_TXN_MAX_SZ + 8));
    b.codes.resize(t->cfg.batch_txn_max);
    b.txns.reserve(t->cfg.batch_txn_max);
    b.items.reserve(t->cfg.batch_txn_max);
    t->pool.push_back(&b);
  }
  return t;
}

void fdgpu_vtile_delete(fdgpu_vtile_t *t) {
  if (!t) return;
  /* drain: the verifier may still write codes into in-flight batches */
  for (Batch *b : t->inflight) {
    if (!b->done) {
      if (b->staged) t->ver.poll_keep(t->ver.ctx, b->ticket, b->codes.data(), 1);
      else t->ver.poll(t->ver.ctx, b->ticket, b->codes.data(), 1);
    }
    if (b->staged) t->ver.release(t->ver.ctx, b->ticket);
  }
  if (t->open && t->open->staged && t->ver.stage_cancel) t->ver.stage_cancel(t->ver.ctx);
  delete t;
}

int64_t fdgpu_vtile_step(fdgpu_vtile_t *t) {
  const int64_t n = t->resolve();
  if (n < 0) return n;
  t->ingest();
  const int rc = t->submit(false);
  if (rc < 0) return rc;
  return n;
}

int fdgpu_vtile_flush(fdgpu_vtile_t *t) {
  int rc = t->submit(true);
  while (rc == 0 && t->open && !t->open->items.empty()) {   /* wait for a free in-flight slot */
    const int64_t n = t->resolve();
    if (n < 0) return (int)n;
    rc = t->submit(true);
  }
  if (rc < 0) return rc;
  while (!t->inflight.empty()) {
    Batch *b = t->inflight.front();
    if (!b->done) {
      const int r = b->staged ? t->ver.poll_keep(t->ver.ctx, b->ticket, b->codes.data(), 1)
                              : t->ver.poll(t->ver.ctx, b->ticket, b->codes.data(), 1);
      if (r != FDGPU_OK) return r;
      b->done = true;
    }
    const int64_t n = t->resolve();
    if (n < 0) return (int)n;
    if (!t->inflight.empty() && t->inflight.front() == b) return FDGPU_ERR_FULL;   /* out-link credits exhausted */
  }
  return 0;
}

int fdgpu_vtile_run(fdgpu_vtile_t *t, uint64_t in_frags, double timeout_s) {
  const uint64_t t0 = now_ns(), lim = (uint64_t)(timeout_s * 1e9);
  uint64_t idle = 0;
  while (t->rx_seq - t->cfg.in_seq0 < in_frags) {
    const uint64_t before = t->rx_seq;
    const int64_t n = fdgpu_vtile_step(t);
    if (n < 0) return (int)n;
    if (t->rx_seq == before && n == 0) {
      /* nothing new: push out a partial batch rather than wait */
      if (++idle > 64) { const int rc = t->submit(true); if (rc < 0) return rc; idle = 0; }
      if (now_ns() - t0 > lim) return FDGPU_ERR_FULL;
    } else {
      idle = 0;
    }
  }
  return fdgpu_vtile_flush(t);
}

void fdgpu_vtile_stats(const fdgpu_vtile_t *t, fdgpu_vtile_stats_t *out) {
  *out = t->st;
  out->lat_cnt = t->lat.size();
}

uint64_t fdgpu_vtile_latencies(const fdgpu_vtile_t *t, uint64_t *out, uint64_t max) {
  const uint64_t n = std::min<uint64_t>(max, t->lat.size());
  std::memcpy(out, t->lat.data(), n * 8);
  return n;
}

void *fdgpu_vtile_tcache(fdgpu_vtile_t *t) { return t->tcache; }

void fdgpu_vtile_log_enable(fdgpu_vtile_t *t, uint64_t log_max) {
  t->log_max = log_max;
  t->log_seq.reserve(log_max);
  t->log_code.reserve(log_max);
}

uint64_t fdgpu_vtile_log(const fdgpu_vtile_t *t, uint64_t *seqs, int8_t *codes, uint64_t max) {
  const uint64_t n = std::min<uint64_t>(max, t->log_seq.size());
  std::memcpy(seqs, t->log_seq.data(), n * 8);
  std::memcpy(codes, t->log_code.data(), n);
  return n;
}

}  // extern "C"

/* --------------------------------------------------------- dedup tile */

/* The dedup tile's tcache at the reference's depth is a 64 MB map + a 32 MB
   ring that every frag touches at random: on 4 KB pages each probe also
   misses the TLB, so the region asks for transparent huge pages (anonymous
   THP is madvise-only on the hosts measured).  A forked child re-homes it
   into memory of its own before entering the sandbox (fdgpu_dtile_rehome): a
   copy-on-write huge page would be split on the child's first write. */
namespace {
struct huge_region {
  void *map = nullptr;
  size_t len = 0;
  void *base = nullptr;
};
constexpr size_t HUGE_SZ = 2ull << 20;
huge_region huge_alloc(size_t bytes) {
  huge_region r;
  r.len = (bytes + 2 * HUGE_SZ - 1) & ~(HUGE_SZ - 1);
  r.map = mmap(nullptr, r.len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (r.map == MAP_FAILED) return huge_region{};
  r.base = (void *)(((uintptr_t)r.map + HUGE_SZ - 1) & ~(uintptr_t)(HUGE_SZ - 1));
  (void)madvise(r.base, bytes, MADV_HUGEPAGE);     /* a hint: 4 KB pages if the host offers none */
  return r;
}
void huge_free(huge_region &r) {
  if (r.map) munmap(r.map, r.len);
  r = huge_region{};
}
}  // namespace

struct fdgpu_dtile {
  fdgpu_dtile_cfg_t cfg{};
  huge_region tc_mem;
  uint64_t tc_bytes = 0;
  void *tcache = nullptr;
  uint64_t rx_seq[16] = {};
  uint64_t fseq_pub[16] = {};          /* what the tile last stored into each in link's fseq */
  uint64_t out_seq = 0, out_chunk = 0;
  uint32_t next_in = 0;
  fdgpu_dtile_stats_t st{};
};

extern "C" {

fdgpu_dtile_t *fdgpu_dtile_new(const fdgpu_dtile_cfg_t *cfg) {
  if (!cfg || !cfg->in_cnt || cfg->in_cnt > 16 || !cfg->out_mcache || !cfg->out_base || !cfg->tcache_depth)
    return nullptr;
  auto *t = new (std::nothrow) fdgpu_dtile;
  if (!t) return nullptr;
  t->cfg = *cfg;
  const uint64_t fp = fdt_tcache_footprint(cfg->tcache_depth, cfg->tcache_map_cnt);
  if (!fp) { delete t; return nullptr; }
  t->tc_mem = huge_alloc(fp);
  if (!t->tc_mem.base) { delete t; return nullptr; }
  t->tc_bytes = fp;
  t->tcache = fdt_tcache_new(t->tc_mem.base, cfg->tcache_depth, cfg->tcache_map_cnt);
  for (uint32_t i = 0; i < cfg->in_cnt; i++) t->rx_seq[i] = t->fseq_pub[i] = cfg->in_seq0[i];
  t->out_seq = cfg->out_seq0;
  t->out_chunk = cfg->out_chunk0;
  return t;
}

void fdgpu_dtile_delete(fdgpu_dtile_t *t) {
  if (!t) return;
  huge_free(t->tc_mem);
  delete t;
}

int fdgpu_dtile_rehome(fdgpu_dtile_t *t) {
  huge_region r = huge_alloc(t->tc_bytes);
  if (!r.base) return -1;
  std::memcpy(r.base, t->tc_mem.base, t->tc_bytes);
  t->tc_mem = r;                      /* the old mapping stays (shared with the parent until it exits) */
  t->tcache = r.base;
  return 0;
}

/* One pass over the in links, at most one frag from each (the mux's
   round-robin service order), fd_dedup.c:89-205. */
int64_t fdgpu_dtile_step(fdgpu_dtile_t *t) {
  const fdgpu_dtile_cfg_t &c = t->cfg;
  int64_t n = 0;
  uint32_t tspub = 0;
  for (uint32_t k = 0; k < c.in_cnt; k++) {
    const uint32_t i = (t->next_in + k) % c.in_cnt;
    fdt_frag_meta_t m;
    uint64_t found;
    const int rc = fdt_mcache_poll(c.in_mcache[i], c.in_depth[i], t->rx_seq[i], &m, &found);
    if (rc == 0) continue;
    if (rc < 0) { t->st.overrun += found - t->rx_seq[i]; t->rx_seq[i] = found; continue; }
    const uint64_t seq = t->rx_seq[i]++;
    {
      /* the frag 4 seqs on, if out already: its payload into the cache now
         (the copy below is latency-bound on payloads the GPU wrote to host
         memory), and the line 8 on */
      const uint64_t mask = c.in_depth[i] - 1;
      const fdt_frag_meta_t *nl = c.in_mcache[i] + ((seq + 4) & mask);
      if (__atomic_load_n(&nl->seq, __ATOMIC_RELAXED) == seq + 4 && nl->chunk <= c.in_wmark[i]) {
        const uint8_t *np = c.in_base[i] + ((uint64_t)nl->chunk << FDT_CHUNK_LG_SZ);
        const uint32_t nsz = nl->sz < FDT_TPU_DCACHE_MTU ? nl->sz : FDT_TPU_DCACHE_MTU;
        for (uint32_t o = 0; o < nsz; o += 64) __builtin_prefetch(np + o);
      }
      __builtin_prefetch(c.in_mcache[i] + ((seq + 8) & mask));
      /* the tcache lines of the insert two frags on (its tag, from the payload
         prefetched two steps ago: a hint only, every value re-read below) and
         of the tag the insert after it evicts: each a random line of a map
         that outgrows every cache at the reference's depth */
      if (i >= c.unparsed_in_cnt) {
        const fdt_frag_meta_t *ml = c.in_mcache[i] + ((seq + 2) & mask);
        const uint64_t msq = __atomic_load_n(&ml->seq, __ATOMIC_RELAXED);
        const uint64_t mch = ml->chunk, msz = ml->sz;
        if (msq == seq + 2 && mch >= c.in_chunk0[i] && mch <= c.in_wmark[i] && msz >= 2 && msz <= FDT_TPU_DCACHE_MTU) {
          const uint8_t *mp = c.in_base[i] + (mch << FDT_CHUNK_LG_SZ);
          uint16_t psz;
          std::memcpy(&psz, mp + msz - 2, 2);
          if (align2(psz) + sizeof(fdt_txn_t) + 2 <= msz) {
            uint16_t so;
            std::memcpy(&so, mp + align2(psz) + offsetof(fdt_txn_t, signature_off), 2);
            if ((uint64_t)so + 64 <= msz) fdt_tcache_prefetch(t->tcache, fdt_hash(c.hashmap_seed, mp + so, 64));
          }
        }
        fdt_tcache_prefetch_evict(t->tcache, 3);
      }
    }
    t->st.in_frags++;
    n++;
    if (m.chunk < c.in_chunk0[i] || m.chunk > c.in_wmark[i] || m.sz > FDT_TPU_DCACHE_MTU) { t->st.corrupt++; continue; }
    uint8_t *dst = c.out_base + (t->out_chunk << FDT_CHUNK_LG_SZ);
    std::memcpy(dst, c.in_base[i] + ((uint64_t)m.chunk << FDT_CHUNK_LG_SZ), m.sz);
    if (fdt_mcache_query(c.in_mcache[i], c.in_depth[i], seq) != seq) { t->st.overrun++; continue; }
    uint64_t sz = m.sz;
    const fdt_txn_t *txn;
    if (i < c.unparsed_in_cnt) {
      /* raw txn (gossip): parse into the trailer like the verify tile */
      const uint64_t toff = align2(sz);
      if (toff > FDT_TPU_DCACHE_MTU - FDT_TXN_MAX_SZ - 2) { t->st.parse_fail++; continue; }
      const uint64_t tsz = fdt_txn_parse(dst, sz, dst + toff, nullptr);
      if (!tsz) { t->st.parse_fail++; continue; }
      const uint16_t psz = (uint16_t)sz;
      std::memcpy(dst + toff + tsz, &psz, 2);
      txn = (const fdt_txn_t *)(dst + toff);
      sz = toff + tsz + 2;
    } else {
      if (sz < 2) { t->st.corrupt++; continue; }
      uint16_t psz;
      std::memcpy(&psz, dst + sz - 2, 2);
      if (align2(psz) + sizeof(fdt_txn_t) + 2 > sz) { t->st.corrupt++; continue; }
      txn = (const fdt_txn_t *)(dst + align2(psz));
    }
    if ((uint64_t)txn->signature_off + 64 > sz) { t->st.corrupt++; continue; }
    const uint64_t tag = fdt_hash(c.hashmap_seed, dst + txn->signature_off, 64);
    if (fdt_tcache_insert(t->tcache, tag)) { t->st.dup++; continue; }
    if (!tspub) tspub = (uint32_t)now_ns() | 1u;            /* one clock read per pass, not per frag */
    fdt_mcache_publish(c.out_mcache, c.out_depth, t->out_seq, 0, t->out_chunk, sz, m.ctl, m.tsorig, tspub);
    t->out_seq++;
    t->out_chunk = fdt_dcache_compact_next(t->out_chunk, sz, c.out_chunk0, c.out_wmark);
    t->st.published++;
  }
  /* reliable links: every frag this pass took is copied out, so its line
     and chunk may be reused -- publish the progress (fd_fseq_update) */
  for (uint32_t i = 0; i < c.in_cnt; i++)
    if (c.in_fseq[i] && t->fseq_pub[i] != t->rx_seq[i]) {   /* (an unchanged value is not re-stored: the line is shared) */
      __atomic_store_n(c.in_fseq[i], t->rx_seq[i], __ATOMIC_RELEASE);
      t->fseq_pub[i] = t->rx_seq[i];
    }
  t->next_in = (t->next_in + 1) % c.in_cnt;
  return n;
}

void fdgpu_dtile_stats(const fdgpu_dtile_t *t, fdgpu_dtile_stats_t *out) { *out = t->st; }

void *fdgpu_dtile_tcache(fdgpu_dtile_t *t) { return t ? t->tcache : nullptr; }

}  // extern "C"

/* ------------------------------------------------------------ producer */

struct fdgpu_producer {
  std::thread th;
  std::atomic<uint64_t> published{0};
  std::atomic<int> done{0};
  double elapsed = 0;
};

extern "C" {

fdgpu_producer_t *fdgpu_producer_start(fdt_frag_meta_t *mcache, uint64_t depth, uint64_t seq0, uint8_t *base,
                                       uint64_t chunk0, uint64_t wmark, const uint8_t *arena, const uint64_t *off,
                                       const uint32_t *sz, uint64_t cnt, double rate_tps) {
  if (!mcache || !base || !arena || !off || !sz || !depth || (depth & (depth - 1))) return nullptr;
  auto *p = new (std::nothrow) fdgpu_producer;
  if (!p) return nullptr;
  p->th = std::thread([=]() {
    /* pacing and the frag timestamps run on the cycle counter (the
       reference stamps frags with fd_tickcount): a clock_gettime per frag
       is a sizeable share of an 80-ns frag budget */
    const uint64_t c0 = tick(), t0 = now_ns();
    double ticks_per_ns = 1.0;
    if (rate_tps > 0) {
      while (now_ns() - t0 < 2000000) {}                /* 2 ms calibration of the counter */
      ticks_per_ns = (double)(tick() - c0) / (double)(now_ns() - t0);
    }
    const double ticks_per_frag = rate_tps > 0 ? ticks_per_ns * 1e9 / rate_tps : 0.0;
    const uint64_t p0 = tick(), t_pub0 = now_ns();       /* publishing starts (the calibration is not counted) */
    uint64_t chunk = chunk0;
    const uint16_t ctl = (uint16_t)fdt_frag_meta_ctl(0, 1, 1, 0);
    for (uint64_t i = 0; i < cnt; i++) {
      if (i + 8 < cnt) {                                /* the source is cold: stream it in ahead */
        const uint8_t *q = arena + off[i + 8];
        for (uint32_t k = 0; k < sz[i + 8]; k += 64) __builtin_prefetch(q + k);
      }
      if (rate_tps > 0) {
        const uint64_t due = p0 + (uint64_t)((double)i * ticks_per_frag);
        while (tick() < due) { /* spin: sub-microsecond pacing */ }
      }
      const uint32_t n = std::min<uint32_t>(sz[i], (uint32_t)FDT_TPU_MTU);
      std::memcpy(base + (chunk << FDT_CHUNK_LG_SZ), arena + off[i], n);
      const uint32_t ts = (uint32_t)tick();
      fdt_mcache_publish(mcache, depth, seq0 + i, 0, chunk, n, ctl, ts, ts);
      chunk = fdt_dcache_compact_next(chunk, n, chunk0, wmark);
      if ((i & 255) == 255 || i + 1 == cnt) p->published.store(i + 1, std::memory_order_relaxed);
    }
    p->elapsed = (double)(now_ns() - t_pub0) * 1e-9;
    p->done.store(1, std::memory_order_release);
  });
  return p;
}

int fdgpu_producer_done(const fdgpu_producer_t *p) { return p ? p->done.load(std::memory_order_acquire) : 1; }

uint64_t fdgpu_producer_join(fdgpu_producer_t *p, double *elapsed_s) {
  if (!p) return 0;
  p->th.join();
  const uint64_t n = p->published.load();
  if (elapsed_s) *elapsed_s = p->elapsed;
  delete p;
  return n;
}

}  // extern "C"
