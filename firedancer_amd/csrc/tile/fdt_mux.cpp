/* fdt_mux.cpp -- the reference's mux tile API restated (fdt_mux_run,
   fdt_mux_publish: src/disco/mux/fd_mux.h:106-299,484-496 and the run loop
   of fd_mux.c:387-699), and the batched GPU verify tile written as mux
   callbacks (fdgpu_vmux_*: fd_verify.c:36-148,232-246).  See
   include/fd_verify_tile.h for the contract. */
#include <immintrin.h>
#include <time.h>

#include <sys/syscall.h>
#include <unistd.h>
#include <x86intrin.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstddef>
#include <cstring>
#include <deque>
#include <new>
#include <vector>

#include "../../../include/fd_verify_tile.h"
#include "../fdt_parse.h"

namespace {

inline uint64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}
inline uint64_t ld_acq(const uint64_t *p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline void st_rel(uint64_t *p, uint64_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }
inline bool pow2(uint64_t x) { return x && !(x & (x - 1)); }
inline uint64_t align2(uint64_t x) { return (x + 1) & ~1ull; }

/* the time stamp counter's rate, measured once per process (the reference's
   fd_tempo_tick_per_ns) */
double tick_per_ns() {
  static double r = [] {
    const uint64_t c0 = __rdtsc(), t0 = now_ns();
    while (now_ns() - t0 < 2000000) {}
    return (double)(__rdtsc() - c0) / (double)(now_ns() - t0);
  }();
  return r;
}

/* the loop's metrics as fd_mux.c keeps them: histograms sampled every
   iteration, link counters accumulated locally and drained at housekeeping */
struct MuxMetrics {
  fdt_mux_metrics_t *out;
  fdt_mux_metrics_t m;
  uint64_t now;
  bool in_backp = false;
  explicit MuxMetrics(fdt_mux_metrics_t *o) : out(o) {
    std::memset(&m, 0, sizeof m);
    if (!out) return;
    const double tpn = tick_per_ns();
    const uint64_t t50ns = (uint64_t)(50.0 * tpn), t50us = (uint64_t)(50000.0 * tpn);
    for (fdt_histf_t *h : {&m.loop_housekeeping_duration_ticks, &m.loop_backpressure_duration_ticks,
                           &m.loop_caught_up_duration_ticks, &m.loop_overrun_polling_duration_ticks,
                           &m.loop_overrun_reading_duration_ticks, &m.loop_filter_before_fragment_duration_ticks,
                           &m.loop_filter_after_fragment_duration_ticks, &m.loop_finish_duration_ticks})
      fdt_histf_init(h, t50ns, t50us);
    fdt_histf_init(&m.fragment_filtered_size_bytes, 0, 2094);     /* metrics.xml: min 0, max 2094 */
    fdt_histf_init(&m.fragment_handled_size_bytes, 0, 2094);
    m.tick_per_ns = tpn;
    m.tile_pid = (uint64_t)getpid();
    m.tile_tid = (uint64_t)syscall(SYS_gettid);
    now = __rdtsc();
  }
  /* one loop iteration ended: its duration into h */
  void lap(fdt_histf_t &h) {
    if (!out) return;
    const uint64_t next = __rdtsc();
    fdt_histf_sample(&h, next - now);
    now = next;
  }
  /* k loop iterations ended at once: k samples, each a k-th of the time */
  void lap_n(fdt_histf_t &h, uint64_t k) {
    if (!out) return;
    const uint64_t next = __rdtsc(), d = (next - now) / k;
    for (uint64_t j = 0; j < k; j++) fdt_histf_sample(&h, d);
    now = next;
  }
  /* a seqlock over the shared copy: its housekeeping_cnt is odd while a
     write is under way and twice the writes so far once it is done; the
     words go out as relaxed atomic stores, so an observer that reads the
     count, copies and re-reads it gets a consistent snapshot or retries */
  void write() {
    if (!out) return;
    const uint64_t k = ++m.housekeeping_cnt;
    uint64_t *seq = &out->housekeeping_cnt;
    __atomic_store_n(seq, 2 * k - 1, __ATOMIC_RELAXED);
    std::atomic_thread_fence(std::memory_order_release);
    static_assert(sizeof m % 8 == 0 && offsetof(fdt_mux_metrics_t, housekeeping_cnt) + 8 == sizeof m,
                  "the sequence word is the last");
    const uint64_t *src = (const uint64_t *)&m;
    uint64_t *dst = (uint64_t *)out;
    for (size_t w = 0; w + 1 < sizeof m / 8; w++) __atomic_store_n(dst + w, src[w], __ATOMIC_RELAXED);
    __atomic_store_n(seq, 2 * k, __ATOMIC_RELEASE);
  }
};

}  // namespace

/* ------------------------------------------------------------------ mux */

namespace {

/* the vmux tile's own instance of the loop (below, after its callbacks) */
bool is_vmux_callbacks(const fdt_mux_callbacks_t *cb);
int vmux_loop(const fdt_mux_cfg_t *cfg, void *ctx, const volatile uint64_t *halt, fdt_mux_stats_t *stats_out);

/* the loop's calls out: through the callback table (any tile) ... */
struct CbHooks {
  const fdt_mux_callbacks_t *cb;
  void *ctx;
  void metrics_write() { if (cb->metrics_write) cb->metrics_write(ctx); }
  void during_housekeeping() { if (cb->during_housekeeping) cb->during_housekeeping(ctx); }
  void before_credit(fdt_mux_context_t *m) { if (cb->before_credit) cb->before_credit(ctx, m); }
  void after_credit(fdt_mux_context_t *m, int *p) { if (cb->after_credit) cb->after_credit(ctx, m, p); }
  uint64_t skip(uint64_t, uint64_t) { return 0; }
  void skipped(uint64_t, uint64_t, uint64_t) {}
  void caught_up(uint64_t) {}
  bool has_before_frag() const { return cb->before_frag != nullptr; }
  void before_frag(uint64_t i, uint64_t seq, uint64_t sig, int *f) { cb->before_frag(ctx, i, seq, sig, f); }
  void during_frag(uint64_t i, uint64_t seq, uint64_t sig, uint64_t chunk, uint64_t sz, int *f) {
    if (cb->during_frag) cb->during_frag(ctx, i, seq, sig, chunk, sz, f);
  }
  void after_frag(uint64_t i, uint64_t seq, uint64_t *sig, uint64_t *chunk, uint64_t *sz, uint64_t *tsorig, int *f,
                  fdt_mux_context_t *m) {
    if (cb->after_frag) cb->after_frag(ctx, i, seq, sig, chunk, sz, tsorig, f, m);
  }
};

template <class H>
int mux_loop(const fdt_mux_cfg_t *cfg, H &h, const volatile uint64_t *halt, fdt_mux_stats_t *stats_out) {
  if (cfg->in_cnt > FDT_MUX_IN_MAX || cfg->out_cnt > FDT_MUX_OUT_MAX) return -1;
  const uint64_t in_cnt = cfg->in_cnt, out_cnt = cfg->out_cnt, flags = cfg->flags;
  const bool copy = (flags & FDT_MUX_FLAG_COPY) != 0;
  uint64_t min_in_depth = UINT64_MAX;
  for (uint64_t i = 0; i < in_cnt; i++) {
    if (!cfg->in_mcache[i] || !pow2(cfg->in_depth[i])) return -1;
    min_in_depth = std::min(min_in_depth, cfg->in_depth[i]);
  }
  /* out stream (fd_mux.c:209-219: no mcache -> a 128-deep dummy, no consumers) */
  fdt_frag_meta_t *mcache = cfg->out_mcache;
  const uint64_t depth = mcache ? cfg->out_depth : 128;
  if (mcache && !pow2(depth)) return -1;
  if (!mcache && out_cnt) return -1;
  for (uint64_t j = 0; j < out_cnt; j++) if (!cfg->out_fseq[j]) return -1;
  /* credits (fd_mux.c:326-335) */
  const uint64_t cr_max_max = copy ? depth : std::min(min_in_depth, depth);
  const uint64_t cr_max = cfg->cr_max ? cfg->cr_max : cr_max_max;
  if (cr_max < 1 || cr_max > cr_max_max) return -1;
  const uint64_t burst = cfg->burst ? cfg->burst : 1;
  const uint64_t lazy = cfg->lazy_iters ? cfg->lazy_iters : 16;

  uint64_t in_seq[FDT_MUX_IN_MAX], out_seq[FDT_MUX_OUT_MAX];
  for (uint64_t i = 0; i < in_cnt; i++) in_seq[i] = cfg->in_seq0[i];
  for (uint64_t j = 0; j < out_cnt; j++) out_seq[j] = ld_acq(cfg->out_fseq[j]);
  uint64_t seq = cfg->out_seq0, cr_avail = 0, cr_filt = 0, in_rr = 0;
  fdt_mux_stats_t st{};
  MuxMetrics mx(cfg->metrics);
  fdt_mux_metrics_t &M = mx.m;
  for (uint64_t hk = 0;; hk--) {
    st.loops++;
    if (!hk) {
      hk = lazy;
      /* housekeeping (fd_mux.c:391-491): receive credits from the outs, send
         our position to the ins, metrics, user callbacks, halt (the cnc signal) */
      for (uint64_t j = 0; j < out_cnt; j++) out_seq[j] = ld_acq(cfg->out_fseq[j]);
      const uint64_t exposed = copy ? 0 : cr_max - cr_avail + cr_filt;
      for (uint64_t i = 0; i < in_cnt; i++) if (cfg->in_fseq[i]) st_rel(cfg->in_fseq[i], in_seq[i] - exposed);
      M.stem_in_backpressure = mx.in_backp;
      mx.write();
      h.metrics_write();
      if (halt && *halt) break;
      if (cr_avail < cr_max) {
        cr_avail = cr_max;
        for (uint64_t j = 0; j < out_cnt; j++) {
          const int64_t lag = std::max<int64_t>((int64_t)(seq - out_seq[j]), 0);
          const uint64_t out_cr = (uint64_t)std::max<int64_t>((int64_t)cr_max - lag, 0);
          cr_avail = std::min(cr_avail, out_cr);
        }
        if (cr_avail == cr_max) cr_filt = 0;
      }
      h.during_housekeeping();
      mx.lap(M.loop_housekeeping_duration_ticks);
    }

    fdt_mux_context_t mux = {mcache, depth, &cr_avail, &seq, out_cnt ? 1ull : 0ull};
    h.before_credit(&mux);
    if (cr_avail < cr_filt + burst) {                                   /* fd_mux.c:548-556 */
      st.backpressure++;
      M.stem_backpressure_count += (uint64_t)!mx.in_backp;              /* transitions into backpressure */
      mx.in_backp = true;
      mx.lap(M.loop_backpressure_duration_ticks);
      continue;
    }
    mx.in_backp = false;
    int poll_in = 1;
    h.after_credit(&mux, &poll_in);
    if (!poll_in || !in_cnt) { mx.lap(M.loop_finish_duration_ticks); continue; }

    const uint64_t i = in_rr;
    in_rr = in_rr + 1 == in_cnt ? 0 : in_rr + 1;
    /* a filter that is a pure function of the seq (the verify tiles' round
       robin, fd_verify.c:46) names the seqs it would drop: the loop reads the
       line of the first seq it keeps, and when that one is published, so are
       the ones before it -- they are filtered as the reference filters them
       one loop each (fd_mux.c:612-624), without their lines */
    const uint64_t skip = h.skip(i, in_seq[i]);
    const uint64_t s_next = in_seq[i] + skip;
    const fdt_frag_meta_t *line = cfg->in_mcache[i] + (s_next & (cfg->in_depth[i] - 1));
    /* the line 16 frags ahead: a tile that reads every frag's line streams
       the whole mcache */
    __builtin_prefetch(cfg->in_mcache[i] + ((s_next + 16) & (cfg->in_depth[i] - 1)));
    const uint64_t seq_found = ld_acq(&line->seq);
    const int64_t diff = (int64_t)(s_next - seq_found);
    if (diff) {                                     /* caught up, or overrun (fd_mux.c:595-609) */
      if (diff < 0) {
        const uint64_t lost = seq_found - in_seq[i];
        st.overrun_polling += lost;
        M.link_in[i].overrun_polling_count++;
        M.link_in[i].overrun_polling_frag_count += lost;
        in_seq[i] = seq_found;
        mx.lap(M.loop_overrun_polling_duration_ticks);
      } else if (skip) {
        /* the kept seq is not out yet: filter the skipped ones that are (the
           last ones of a stream have no kept seq after them) */
        const uint64_t mask = cfg->in_depth[i] - 1;
        const uint64_t k = ld_acq(&cfg->in_mcache[i][(s_next - 1) & mask].seq) == s_next - 1 ? skip
                         : ld_acq(&cfg->in_mcache[i][in_seq[i] & mask].seq) == in_seq[i] ? 1 : 0;
        if (k) {
          h.skipped(i, in_seq[i], k);
          if (!copy) cr_filt += k * (uint64_t)(cr_avail < cr_max);
          st.in_frags += k;
          st.filtered_before += k;
          in_seq[i] += k;
          mx.lap_n(M.loop_filter_before_fragment_duration_ticks, k);
        } else {
          h.caught_up(i);
          mx.lap(M.loop_caught_up_duration_ticks);
        }
      } else {
        h.caught_up(i);
        mx.lap(M.loop_caught_up_duration_ticks);
      }
      continue;
    }
    if (skip) {
      h.skipped(i, in_seq[i], skip);
      if (!copy) cr_filt += skip * (uint64_t)(cr_avail < cr_max);
      st.in_frags += skip;
      st.filtered_before += skip;
      mx.lap_n(M.loop_filter_before_fragment_duration_ticks, skip);
      in_seq[i] = s_next;
    }
    uint64_t sig = line->sig;
    st.in_frags++;
    if (h.has_before_frag()) {
      int filter = 0;
      h.before_frag(i, seq_found, sig, &filter);
      if (filter) {
        if (!copy) cr_filt += (uint64_t)(cr_avail < cr_max);
        in_seq[i]++;
        st.filtered_before++;
        mx.lap(M.loop_filter_before_fragment_duration_ticks);
        continue;
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    uint64_t chunk = line->chunk, sz = line->sz;
    const uint64_t ctl = line->ctl, tsorig = line->tsorig;
    std::atomic_thread_fence(std::memory_order_acquire);
    const uint64_t seq_test = ld_acq(&line->seq);
    int filter = 0;
    h.during_frag(i, seq_found, sig, chunk, sz, &filter);
    /* the reference checks the seq read before during_frag (fd_mux.c:641-655);
       the quic -> verify link has no backpressure, so the payload copy is
       checked too */
    const uint64_t seq_test2 = ld_acq(&line->seq);
    if (seq_test != seq_found || seq_test2 != seq_found) {
      st.overrun_reading++;
      M.link_in[i].overrun_reading_count++;
      in_seq[i] = seq_test2;
      mx.lap(M.loop_overrun_reading_duration_ticks);
      continue;
    }
    uint64_t out_sz = sz, out_tsorig = tsorig;
    if (!filter) h.after_frag(i, seq_found, &sig, &chunk, &out_sz, &out_tsorig, &filter, &mux);
    if (filter) {
      if (!copy) cr_filt += (uint64_t)(cr_avail < cr_max);
      st.filtered_after++;
    } else if (!(flags & FDT_MUX_FLAG_MANUAL_PUBLISH)) {
      fdt_mux_publish(&mux, sig, chunk, out_sz, ctl, out_tsorig, (uint32_t)now_ns());
      st.published++;
    }
    in_seq[i]++;
    /* fd_mux.c:690-697: PublishedCount/Size or FilteredCount/Size of the in link */
    fdt_link_in_metrics_t &L = M.link_in[i];
    if (filter) { L.filtered_count++; L.filtered_size_bytes += sz; }
    else        { L.published_count++; L.published_size_bytes += sz; }
    if (mx.out) {
      mx.lap(filter ? M.loop_filter_after_fragment_duration_ticks : M.loop_finish_duration_ticks);
      fdt_histf_sample(filter ? &M.fragment_filtered_size_bytes : &M.fragment_handled_size_bytes, sz);
    }
  }
  /* halting (fd_mux.c:701-714): every exposed frag counts as consumed */
  for (uint64_t i = 0; i < in_cnt; i++) if (cfg->in_fseq[i]) st_rel(cfg->in_fseq[i], in_seq[i]);
  mx.write();
  if (stats_out) *stats_out = st;
  return 0;
}

}  // namespace


extern "C" {

void fdt_histf_init(fdt_histf_t *h, uint64_t min, uint64_t max) {
  /* fd_histf_new (fd_histf.h:77-117): min >= 1, at least one value per
     bucket, edges ~ min * z^i with max ~ min * z^14 */
  std::memset(h, 0, sizeof *h);
  min = std::max<uint64_t>(min, 1);
  max = std::max<uint64_t>(max, min + FDT_HISTF_BUCKET_CNT - 2);
  h->left_edge[0] = 0;
  h->left_edge[1] = min;
  for (uint64_t i = 2; i < FDT_HISTF_BUCKET_CNT - 1; i++) {
    uint64_t le = (uint64_t)(0.5 + (double)h->left_edge[i - 1] *
                                       std::pow((double)max / (double)h->left_edge[i - 1],
                                                1.0 / (double)(FDT_HISTF_BUCKET_CNT - i)));
    le = std::max(le, h->left_edge[i - 1] + 1);
    h->left_edge[i] = le;
  }
  h->left_edge[FDT_HISTF_BUCKET_CNT - 1] = max;
  h->left_edge[FDT_HISTF_BUCKET_CNT] = UINT64_MAX;
}

void fdt_histf_sample(fdt_histf_t *h, uint64_t v) {
  h->sum += v;
  uint64_t b = FDT_HISTF_BUCKET_CNT - 1;         /* [max, inf) */
  for (uint64_t i = 0; i + 1 < FDT_HISTF_BUCKET_CNT; i++)
    if (v < h->left_edge[i + 1]) { b = i; break; }
  h->counts[b]++;
}

void fdt_mux_publish(fdt_mux_context_t *ctx, uint64_t sig, uint64_t chunk, uint64_t sz, uint64_t ctl,
                     uint64_t tsorig, uint64_t tspub) {
  const uint64_t seq = *ctx->seq;
  fdt_mcache_publish(ctx->mcache, ctx->depth, seq, sig, chunk, sz, ctl, tsorig, tspub);
  *ctx->cr_avail -= ctx->cr_decrement_amount;
  *ctx->seq = seq + 1;
}

int fdt_mux_metrics_snapshot(const fdt_mux_metrics_t *src, fdt_mux_metrics_t *dst, uint64_t max_tries) {
  const uint64_t *s = (const uint64_t *)src;
  uint64_t *d = (uint64_t *)dst;
  const size_t nw = sizeof *src / 8;
  for (uint64_t k = 0; k < max_tries; k++) {
    const uint64_t seq0 = __atomic_load_n(&src->housekeeping_cnt, __ATOMIC_ACQUIRE);
    if (seq0 & 1) { _mm_pause(); continue; }
    for (size_t w = 0; w + 1 < nw; w++) d[w] = __atomic_load_n(s + w, __ATOMIC_RELAXED);
    std::atomic_thread_fence(std::memory_order_acquire);
    if (__atomic_load_n(&src->housekeeping_cnt, __ATOMIC_RELAXED) == seq0) {
      dst->housekeeping_cnt = seq0;
      return 0;
    }
  }
  return -1;
}

int fdt_mux_run(const fdt_mux_cfg_t *cfg, const fdt_mux_callbacks_t *cb, void *ctx, const volatile uint64_t *halt,
                fdt_mux_stats_t *stats_out) {
  if (!cfg || !cb) return -1;
  if (is_vmux_callbacks(cb)) return vmux_loop(cfg, ctx, halt, stats_out);
  CbHooks h{cb, ctx};
  return mux_loop(cfg, h, halt, stats_out);
}

}  // extern "C"

/* ------------------------------------------------------------ vmux tile */

namespace {

struct VItem {                       /* a frag of a batch (host / GPU parse; the gather mode keeps fio + tso) */
  uint64_t seq;
  uint64_t tag;         /* fd_hash(seed, signature 0, 64): the dedup tag, taken while the payload is hot */
  uint32_t chunk;       /* where [payload][pad][fd_txn_t][u16 sz] lies in the out dcache */
  uint32_t sz;          /* that frag's size (gpu_parse: the payload's; the trailer is added at publish) */
  uint32_t sig_off;     /* signature 0, from the frag start */
  uint32_t tsorig;
  uint32_t tr_off;      /* gpu_parse: the parsed fd_txn_t's place in the batch's trailer buffer */
  uint32_t tr_cap;      /*            and its footprint (fdt_txn_peek); gather: the out bytes reserved */
};

struct VBatch {
  uint64_t first_chunk = 0;          /* the arena is out_base + first_chunk * 64 ... + end_off */
  uint64_t end_off = 0;
  std::vector<fdgpu_txn_t> txns;
  std::vector<fdgpu_frag_ex_t> frags;  /* gpu_parse: the verifier's view of the items */
  std::vector<uint8_t> trailers;      /* gpu_parse: parsed fd_txn_t records, filled by poll_frags */
  std::vector<fdgpu_frag_io_t> fio;   /* gather: the frags themselves (seq, size, out room, in link), [0, cnt) ... */
  std::vector<uint32_t> tso;          /*   their tsorig, */
  std::vector<uint32_t> lost;         /*   the ones the lap guard found lapped when it copied them, */
  std::vector<uint64_t> tags;         /*   and the verifier's results: dedup tags, */
  std::vector<uint16_t> out_szs;      /*   out frag sizes */
  uint64_t link_first[FDT_MUX_IN_MAX];   /* gather: the oldest seq taken from each in link, */
  uint64_t link_last[FDT_MUX_IN_MAX];    /*   the newest, */
  uint32_t guard_cur[FDT_MUX_IN_MAX];    /*   the lap guard's cursor over the items of each, */
  uint32_t link_mask = 0;                /*   and which links the batch holds frags of */
  uint64_t tr_used = 0;
  std::vector<VItem> items;
  size_t cnt = 0;                     /* frags in the batch (items, or fio in the gather mode) */
  std::vector<int8_t> codes;
  uint64_t sig_cnt = 0;               /* signatures sent (gpu_parse: the frags' upper bound) */
  int64_t ticket = -1;
  bool closed = false;               /* takes no more frags (full, or the cursor wrapped) */
  bool done = false;
  size_t next = 0;                   /* next item to resolve */
  uint64_t t_first = 0, t_submit = 0;
  uint64_t cu_first = 0;              /* the tile's caught_up_cnt when the batch took its first frag */

  void reset() {
    first_chunk = end_off = sig_cnt = tr_used = 0;
    txns.clear(); items.clear(); frags.clear(); lost.clear();     /* fio, tso: sized once, filled to cnt */
    cnt = 0;
    link_mask = 0;
    ticket = -1; closed = done = false; next = 0; t_first = 0;
  }
};

constexpr uint64_t FRAG_CHUNKS = (FDT_TPU_DCACHE_MTU + FDT_CHUNK_SZ - 1) / FDT_CHUNK_SZ;   /* a maximal out frag */

}  // namespace

struct fdgpu_vmux {
  fdgpu_vmux_cfg_t cfg{};
  fdgpu_verifier_t ver{};
  std::vector<uint64_t> tcache_mem;
  void *tcache = nullptr;                 /* fd_tcache (depth > FDT_TAGRING_MAX) ... */
  fdt_tagring_t ring{};                   /* ... or the ring scan (the tile's 16-deep default) */
  bool use_ring = false;
  /* the ring scan inline, over a fixed 16 or 32 slots (the unused ones hold
     the null tag, which no query reaches): AVX2 compares of four tags each,
     OR-ed, one test (the scalar loop the compiler made of it was a serial
     chain of 16 compare-or steps, a fifth of the tile's time) */
  template <int N> static bool ring_hit(const uint64_t *t, uint64_t tag) {
    const __m256i q = _mm256_set1_epi64x((long long)tag);
    __m256i h = _mm256_cmpeq_epi64(_mm256_loadu_si256((const __m256i *)t), q);
#pragma GCC unroll 8
    for (int i = 4; i < N; i += 4) h = _mm256_or_si256(h, _mm256_cmpeq_epi64(_mm256_loadu_si256((const __m256i *)(t + i)), q));
    return !_mm256_testz_si256(h, h);
  }
  bool tc_query(uint64_t tag) const {
    if (!use_ring) return fdt_tcache_query(tcache, tag);
    if (tag == FDT_TCACHE_TAG_NULL) return true;
    return ring.depth <= 16 ? ring_hit<16>(ring.tag, tag) : ring_hit<FDT_TAGRING_MAX>(ring.tag, tag);
  }
  /* insert a tag the query just missed (fdt_tagring_insert without its re-query) */
  void tc_insert(uint64_t tag) {
    if (!use_ring) { (void)fdt_tcache_insert(tcache, tag); return; }
    ring.tag[ring.oldest] = tag;
    ring.oldest = ring.oldest + 1 >= ring.depth ? 0 : ring.oldest + 1;
  }
  std::vector<uint16_t> cap_of;          /* gather: out-frag room by payload size (fdt_frag_fp_bound) */
  uint64_t out_chunk = 0;                 /* write cursor */
  bool room_ok = false;                   /* room() held at the cursor (the live region only shrinks
                                             until the cursor moves, so a yes stays a yes till then) */
  uint64_t rr_mask = 0;                   /* round_robin_cnt - 1 when a power of two, else 0 */
  uint64_t cur_sz = 0;                    /* the frag between during_frag and after_frag */
  bool cur_ok = false;
  uint64_t cur_fp = 0, cur_sc = 0, cur_tag = 0;   /* gpu_parse: its peeked footprint, signature count, tag */
  std::vector<VBatch> storage;
  std::vector<VBatch *> pool;
  std::deque<VBatch *> inflight;          /* submitted, in ingest order, until published */
  uint32_t busy = 0;                      /* ... of which still on the verifier (not polled done) */
  uint32_t sweeps = 0;                    /* resolve calls (rate-limits polling the batches behind the oldest) */
  VBatch *open = nullptr;
  std::vector<uint32_t> pub_chunk;        /* chunk of each recently published out seq */
  uint64_t pub_mask = 0, published_total = 0;
  int error = 0;
  uint32_t calls = 0;                     /* after_credit calls (rate-limits verifier polls) */
  uint64_t due_tsc = 0, stall_max_tick = 0;   /* the every-64th call's time stamp counter, the longest gap */
  uint64_t caught_up_cnt = 0;             /* polls of an in link that found nothing new ... */
  bool sees_caught_up = false;            /* ... counted (the loop's own instance; a callback table: the timer alone) */
  fdgpu_vtile_stats_t st{};
  std::vector<uint64_t> lat;
  fdgpu_link_t links[FDT_MUX_IN_MAX] = {};   /* gather: the in mcaches, re-checked by the device after its read */
  uint64_t lap_span_max = 0, lap_margin = 0;  /* gather: the lap guard (~0: off) */
  uint64_t log_max = 0;
  std::vector<uint64_t> log_seq;
  std::vector<int8_t> log_code;

  bool gpu_parse = false;                /* fd_txn_parse on the GPU (verifier submit_frags / poll_frags) */
  bool gather = false;                   /* ... and the payload copy too (submit_io / poll_io) */
  uint64_t cur_src = 0, cur_in = 0;       /* gather: the frag between during_frag and after_frag */
  uint64_t final_n = 0;                   /* frags whose outcome is final ... */
  std::atomic<uint64_t> final_cnt{0};    /* ... published for other threads (one writer: a store, no RMW) */

  void log(uint64_t seq, int code) {
    if (log_max && log_seq.size() < log_max) { log_seq.push_back(seq); log_code.push_back((int8_t)code); }
    final_cnt.store(++final_n, std::memory_order_release);
  }

  uint8_t *out_laddr(uint64_t chunk) const { return cfg.out_base + (chunk << FDT_CHUNK_LG_SZ); }
  /* the out chunk frag k of batch b lies at */
  uint64_t chunk_of(const VBatch &b, size_t k) const {
    return gather ? b.first_chunk + (b.fio[k].out_off >> FDT_CHUNK_LG_SZ) : b.items[k].chunk;
  }

  /* chunk of the oldest frag that may still be read: published and possibly
     unconsumed (the mux's exposed count), else reserved by an unresolved
     batch item; false when nothing is live */
  bool live_tail(const fdt_mux_context_t *mux, uint64_t &tail) const {
    uint64_t exposed = cfg.cr_max - std::min(cfg.cr_max, *mux->cr_avail);
    exposed = std::min(exposed, published_total);
    if (exposed) { tail = pub_chunk[(*mux->seq - exposed) & pub_mask]; return true; }
    for (const VBatch *b : inflight)
      if (b->next < b->cnt) { tail = chunk_of(*b, b->next); return true; }
    if (open && open->cnt) { tail = open->first_chunk; return true; }
    return false;
  }

  /* room for one maximal frag at the cursor (the live region is [tail, cursor)
     in ring order) */
  bool room(const fdt_mux_context_t *mux) const {
    uint64_t tail;
    if (!live_tail(mux, tail)) return true;
    const uint64_t w = out_chunk;
    if (w > tail) return true;
    if (w == tail) return false;
    return w + FRAG_CHUNKS <= tail;
  }

  /* a non-blocking poll of one submitted batch: 1 done (its results are
     in the batch, its verifier slot is free), 0 pending, -1 error */
  int poll_one(VBatch *b, int *poll_in) {
    /* poll_ns and poll_done_ns are sampled: every 8th poll is timed and
       counts 8 times (two clock reads cost a pending poll more than the poll) */
    const bool timed = !(st.polls++ & 7u);
    const uint64_t p0 = timed ? now_ns() : 0;
    const int rc = gather ? ver.poll_io(ver.ctx, b->ticket, b->codes.data(), b->tags.data(), b->out_szs.data(), 0)
                   : gpu_parse ? ver.poll_frags(ver.ctx, b->ticket, b->codes.data(), b->trailers.data(), 0)
                               : ver.poll(ver.ctx, b->ticket, b->codes.data(), 0);
    if (rc == FDGPU_PENDING) {
      if (timed) st.poll_ns += 8 * (now_ns() - p0);
      return 0;
    }
    const uint64_t p1 = now_ns();
    if (timed) { st.poll_ns += 8 * (p1 - p0); st.poll_done_ns += 8 * (p1 - p0); }
    st.batch_gpu_ns += p1 - b->t_submit;
    if (rc != FDGPU_OK) { error = rc; *poll_in = 0; return -1; }
    b->done = true;
    busy--;
    for (uint32_t k : b->lost) b->codes[k] = (int8_t)FDGPU_CODE_LAPPED;
    if (gather) note_lap_margin(*b);
    return 1;
  }

  /* gather: the batch is done (the device read its payloads before): how
     many more publishes each of its links' oldest frag had left before the
     producer reuses its line.  The link's newest published seq P is found by
     bisection between the batch's newest frag of the link (published) and
     the oldest's line reuse: published_by(s) holds exactly for s <= P. */
  void note_lap_margin(const VBatch &b) {
    for (uint32_t i = 0; i < cfg.in_cnt; i++) {
      if (!(b.link_mask >> i & 1u)) continue;
      const uint64_t reuse = b.link_first[i] + cfg.in_depth[i];     /* publishing this seq overwrites the oldest */
      uint64_t m;
      if (published_by(i, reuse)) {
        m = 0;
      } else {
        uint64_t lo = b.link_last[i], hi = reuse;                    /* published_by(lo), !published_by(hi) */
        while (hi - lo > 1) {
          const uint64_t mid = lo + (hi - lo) / 2;
          if (published_by(i, mid)) lo = mid; else hi = mid;
        }
        m = reuse - 1 - lo;
      }
      st.lap_margin_min = std::min(st.lap_margin_min, m);
    }
  }

  /* tag, tcache, publish -- strictly in ingest order (fd_verify.h:45-89,
     fd_verify.c:138-147).  Batches finish on the GPU out of order (several
     run at once on their own streams): every finished one is polled, which
     frees its verifier slot for the next batch, while publishing waits for
     the oldest. */
  void resolve(fdt_mux_context_t *mux, int *poll_in) {
    if (busy > 1 && !(sweeps++ & 7u))          /* every 8th call: a poll is a runtime call, a slot freed a few us late costs little */
      for (size_t j = 1; j < inflight.size(); j++)
        if (!inflight[j]->done && poll_one(inflight[j], poll_in) < 0) return;
    while (!inflight.empty()) {
      VBatch *b = inflight.front();
      if (!b->done && poll_one(b, poll_in) <= 0) return;
      const uint64_t t_pub = now_ns();
      struct Acc { uint64_t &ns; uint64_t t0; ~Acc() { ns += now_ns() - t0; } } acc{st.publish_ns, t_pub};
      const uint32_t tspub = (uint32_t)t_pub;
      if (!(gather ? resolve_gather(*b, mux, poll_in, tspub) : resolve_items(*b, mux, poll_in, tspub))) return;
      if (lat.size() < (1u << 22) && b->cnt) lat.push_back(now_ns() - b->t_first);
      inflight.pop_front();
      b->reset();
      pool.push_back(b);
    }
  }

  /* host / GPU parse: resolve a polled batch item by item; false when
     credits ran out mid-way (the mux refreshes them, then the rest is
     resolved from b.next -- nothing of the stalled item was inserted yet) */
  bool resolve_items(VBatch &b, fdt_mux_context_t *mux, int *poll_in, uint32_t tspub) {
    const size_t n = b.items.size();
    while (b.next < n) {
      const size_t k = b.next;
      if (gpu_parse && k + 8 < n) {              /* the trailer store of a frag soon published: own the line */
        const VItem &f = b.items[k + 8];
        __builtin_prefetch(out_laddr(f.chunk) + align2(f.sz), 1);
      }
      const VItem &it = b.items[k];
      const int code = b.codes[k];
      if (gpu_parse && (code == FDGPU_CODE_PARSE_FAIL || code == FDGPU_CODE_TRAILER_CAP)) {
        /* not a transaction: filtered before the dedup check (fd_verify.c:
           117-121); a footprint other than the one reserved: a peek / parse
           disagreement, failed without a verdict */
        if (code == FDGPU_CODE_PARSE_FAIL) { st.parse_fail++; log(it.seq, FDGPU_VTILE_LOG_PARSE_FAIL); }
        else { st.verify_errors++; log(it.seq, FD_TXN_VERIFY_FAILED); }
        b.next++;
        continue;
      }
      uint8_t *frag = out_laddr(it.chunk);
      const uint64_t tag = it.tag;
      int outcome;
      if (tc_query(tag)) outcome = FD_TXN_VERIFY_DEDUP;
      else if (code != FD_ED25519_SUCCESS) outcome = FD_TXN_VERIFY_FAILED;
      else outcome = FD_TXN_VERIFY_SUCCESS;
      if (outcome == FD_TXN_VERIFY_SUCCESS) {
        if (mux->cr_decrement_amount && !*mux->cr_avail) {
          *poll_in = 0;
          st.backpressure++;
          return false;
        }
        tc_insert(tag);                          /* not present: the query above missed */
        uint64_t sz = it.sz;
        if (gpu_parse) {                         /* [payload][pad][fd_txn_t][u16 payload_sz] (fd_verify.c:93-136) */
          const uint64_t toff = align2(it.sz);
          if (toff != it.sz) frag[it.sz] = 0;
          std::memcpy(frag + toff, b.trailers.data() + it.tr_off, it.tr_cap);
          const uint16_t psz = (uint16_t)it.sz;
          std::memcpy(frag + toff + it.tr_cap, &psz, 2);
          sz = toff + it.tr_cap + 2;
        }
        pub_chunk[*mux->seq & pub_mask] = it.chunk;
        fdt_mux_publish(mux, tag, it.chunk, sz, 0, it.tsorig, tspub);
        published_total++;
        st.published++;
      } else if (outcome == FD_TXN_VERIFY_DEDUP) {
        st.dedup++;
      } else {
        st.verify_failed++;
      }
      log(it.seq, outcome);
      b.next++;
    }
    return true;
  }

  /* gather: resolve a polled batch from its frag records (the GPU's codes,
     tags and out sizes); false when credits ran out mid-way (the mux
     refreshes them, then the rest is resolved from b.next) */
  bool resolve_gather(VBatch &b, fdt_mux_context_t *mux, int *poll_in, uint32_t tspub) {
    const size_t n = b.cnt;
    while (b.next < n) {
      const size_t k = b.next;
      const fdgpu_frag_io_t &f = b.fio[k];
      const int code = b.codes[k];
      if (code == FDGPU_CODE_LAPPED) {                  /* the producer overwrote it before it was read */
        st.overrun++;
        st.lapped++;
        log(f.seq, FDGPU_VTILE_LOG_LOST);
        b.next++;
        continue;
      }
      if (code == FDGPU_CODE_PARSE_FAIL || code == FDGPU_CODE_TRAILER_CAP) {
        /* not a transaction: filtered before the dedup check (fd_verify.c:117-121);
           a parsed out frag larger than its reservation: failed without a verdict */
        if (code == FDGPU_CODE_PARSE_FAIL) { st.parse_fail++; log(f.seq, FDGPU_VTILE_LOG_PARSE_FAIL); }
        else { st.verify_errors++; log(f.seq, FD_TXN_VERIFY_FAILED); }
        b.next++;
        continue;
      }
      const uint64_t tag = b.tags[k];
      int outcome;
      if (tc_query(tag)) outcome = FD_TXN_VERIFY_DEDUP;
      else if (code != FD_ED25519_SUCCESS) outcome = FD_TXN_VERIFY_FAILED;
      else outcome = FD_TXN_VERIFY_SUCCESS;
      if (outcome == FD_TXN_VERIFY_SUCCESS) {
        if (mux->cr_decrement_amount && !*mux->cr_avail) {
          *poll_in = 0;                                 /* out of credits: resolved again from here */
          st.backpressure++;
          return false;
        }
        tc_insert(tag);
        const uint64_t chunk = b.first_chunk + (f.out_off >> FDT_CHUNK_LG_SZ);
        pub_chunk[*mux->seq & pub_mask] = (uint32_t)chunk;
        fdt_mux_publish(mux, tag, chunk, b.out_szs[k], 0, b.tso[k], tspub);   /* written there by the GPU */
        published_total++;
        st.published++;
      } else if (outcome == FD_TXN_VERIFY_DEDUP) {
        st.dedup++;
      } else {
        st.verify_failed++;
      }
      log(f.seq, outcome);
      b.next++;
    }
    return true;
  }

  /* gather: has in link i's producer published seq s yet?  Its line holds
     s - depth (or older) until then: a signed difference reads the lap. */
  bool published_by(uint32_t i, uint64_t s) const {
    const fdt_frag_meta_t *line = cfg.in_mcache[i] + (s & (cfg.in_depth[i] - 1));
    return (int64_t)(ld_acq(&line->seq) - s) >= 0;
  }

  /* gather, the lap guard: the device reads a payload only after the batch
     is submitted (and re-checks its line then, fdgpu_submit_frags_io), and
     the quic -> verify producer never waits for the tile.  Before a batch
     goes out -- and while it waits for a free slot -- every frag whose line
     the producer will reuse within lap_margin more publishes is copied here
     into its out frag's room, re-checked as the reference re-checks after
     its copy (fd_mux.c:641-655), and handed to the device from there (link
     0: no device re-check).  One line read per link tells whether any frag
     of it is at risk (its oldest frag is the first to be lapped); younger
     frags of a link are safer, so each link's scan stops at its first frag
     not at risk. */
  void lap_guard(VBatch &b) {
    for (uint32_t i = 0; i < cfg.in_cnt; i++) {
      if (!(b.link_mask >> i & 1u)) continue;
      const uint64_t depth = cfg.in_depth[i], m = std::min(lap_margin, depth);
      const size_t n = b.cnt;
      size_t k = b.guard_cur[i];
      while (k < n && b.fio[k].link != i + 1u) k++;
      if (k == n || !published_by(i, b.fio[k].seq + depth - m)) { b.guard_cur[i] = (uint32_t)k; continue; }
      for (; k < n; k++) {
        fdgpu_frag_io_t &f = b.fio[k];
        if (f.link != i + 1u) continue;
        if (!published_by(i, f.seq + depth - m)) break;
        uint8_t *dst = out_laddr(b.first_chunk + (f.out_off >> FDT_CHUNK_LG_SZ));
        std::memcpy(dst, (const void *)(uintptr_t)f.src, f.sz);
        std::atomic_thread_fence(std::memory_order_acquire);
        const fdt_frag_meta_t *line = cfg.in_mcache[i] + (f.seq & (depth - 1));
        if (ld_acq(&line->seq) != f.seq) b.lost.push_back((uint32_t)k);   /* lapped already: may be torn */
        else st.rescued++;
        f.src = (uint64_t)(uintptr_t)dst;                 /* the device reads this copy */
        f.link = 0;
      }
      b.guard_cur[i] = (uint32_t)k;
    }
  }

  /* the verifier refused the batch as malformed: its txns fail (logged),
     nothing is published, the tile goes on (device errors stay fatal) */
  void reject_open() {
    for (size_t k = 0; k < open->cnt; k++) {
      st.verify_errors++;
      log(gather ? open->fio[k].seq : open->items[k].seq, FD_TXN_VERIFY_FAILED);
    }
    open->reset();
    pool.push_back(open);
    open = nullptr;
  }

  void submit() {
    if (!open || !open->cnt) return;
    const uint64_t s0 = now_ns();
    if (gather && lap_margin != ~0ull) lap_guard(*open);    /* also while the batch fills or waits for a slot */
    /* a partial batch goes out once its oldest frag waited batch_wait_ns and
       the tile has since found its in links drained; while frags keep
       coming faster than it reads them, the batch fills (capacity: full
       batches, not a timer's worth) */
    if (!open->closed && (s0 - open->t_first < cfg.batch_wait_ns || (sees_caught_up && caught_up_cnt == open->cu_first)))
      return;
    if (busy >= cfg.inflight_max) return;
    /* timed from before the lap guard's pass; the calls that return above
       (most: one every 64 frags) are not, which saves them a clock read */
    struct Acc {
      uint64_t &ns, &mx; uint64_t t0;
      ~Acc() { const uint64_t d = now_ns() - t0; ns += d; mx = std::max(mx, d); }
    } acc{st.submit_ns, st.submit_max_ns, s0};
    int64_t t;
    if (gather) {
      const size_t n = open->cnt;
      if (open->tags.size() < n) { open->tags.resize(cfg.batch_txn_max); open->out_szs.resize(cfg.batch_txn_max); }
      t = ver.submit_io(ver.ctx, open->fio.data(), n, out_laddr(open->first_chunk), open->end_off, cfg.hashmap_seed,
                        links, cfg.in_cnt);
    } else if (gpu_parse) {
      if (open->trailers.size() < open->tr_used) open->trailers.resize(open->tr_used);
      t = ver.submit_frags(ver.ctx, out_laddr(open->first_chunk), open->end_off, open->frags.data(),
                           open->frags.size(), open->tr_used);
    } else {
      t = ver.submit(ver.ctx, out_laddr(open->first_chunk), open->end_off, open->txns.data(), open->txns.size());
    }
    if (t == FDGPU_ERR_FULL) return;
    if (t == FDGPU_ERR_INVAL) { reject_open(); return; }
    if (t < 0) { error = (int)t; return; }
    open->ticket = t;
    open->t_submit = now_ns();
    st.batch_fill_ns += open->t_submit - open->t_first;
    inflight.push_back(open);
    busy++;
    open = nullptr;
    st.batches++;
  }

  bool can_take() {
    if (open && open->closed) return false;
    if (!open) {
      if (pool.empty()) return false;
      open = pool.back();
      pool.pop_back();
    }
    return true;
  }
};

namespace {

__attribute__((always_inline)) inline void vm_before_frag(void *ctx, uint64_t in_idx, uint64_t seq, uint64_t sig, int *opt_filter) {
  (void)in_idx; (void)sig;
  auto *t = (fdgpu_vmux *)ctx;
  t->st.in_frags++;
  const uint64_t cnt = t->cfg.round_robin_cnt;
  if (cnt > 1 && (t->rr_mask ? (seq & t->rr_mask) : seq % cnt) != t->cfg.round_robin_idx) {
    *opt_filter = 1;
    t->st.filtered_rr++;
    t->log(seq, FDGPU_VTILE_LOG_FILTERED);
  }
}

__attribute__((always_inline)) inline void vm_during_frag(void *ctx, uint64_t in_idx, uint64_t seq, uint64_t sig, uint64_t chunk, uint64_t sz,
                    int *opt_filter) {
  (void)sig;
  auto *t = (fdgpu_vmux *)ctx;
  const fdgpu_vmux_cfg_t &c = t->cfg;
  t->cur_ok = false;
  if (chunk < c.in_chunk0[in_idx] || chunk > c.in_wmark[in_idx] || sz > FDT_TPU_MTU) {
    /* the reference aborts the tile here (FD_LOG_ERR, fd_verify.c:67-68) */
    t->st.corrupt++;
    t->log(seq, FDGPU_VTILE_LOG_LOST);
    *opt_filter = 1;
    return;
  }
  const uint8_t *src = c.in_base[in_idx] + (chunk << FDT_CHUNK_LG_SZ);
  if (t->gather) {                    /* the GPU reads it there (after_credit re-checks the line after the poll) */
    t->cur_src = (uint64_t)(uintptr_t)src;
    t->cur_in = in_idx;
    t->cur_sz = sz;
    t->cur_ok = true;
    return;
  }
  std::memcpy(t->out_laddr(t->out_chunk), src, sz);
  if (t->gpu_parse) {
    /* read the counts and hash signature 0 from the source just copied (in
       L1): the mux's seq re-check after during_frag discards them with the
       frag if the producer overwrote it meanwhile */
    t->cur_fp = fdt_txn_peek(src, sz, &t->cur_sc);
    t->cur_tag = sz >= 65 ? fdt_hash(c.hashmap_seed, src + 1, 64) : 0;
  }
  t->cur_sz = sz;
  t->cur_ok = true;
}

__attribute__((always_inline)) inline void vm_after_frag(void *ctx, uint64_t in_idx, uint64_t seq, uint64_t *opt_sig, uint64_t *opt_chunk,
                   uint64_t *opt_sz, uint64_t *opt_tsorig, int *opt_filter, fdt_mux_context_t *mux) {
  (void)in_idx; (void)opt_sig; (void)opt_chunk; (void)mux;
  auto *t = (fdgpu_vmux *)ctx;
  if (!t->cur_ok) { *opt_filter = 1; return; }
  const uint64_t payload_sz = *opt_sz;
  uint8_t *txn = t->out_laddr(t->out_chunk);
  const uint64_t toff = align2(payload_sz);
  if (t->gather) {
    /* reserve the out frag's room from the size alone (the tile never reads
       the payload); the GPU writes [payload][pad][fd_txn_t][u16] there */
    VBatch &b = *t->open;
    if (!b.cnt) { b.first_chunk = t->out_chunk; b.t_first = now_ns(); b.cu_first = t->caught_up_cnt; }
    const uint64_t off = (t->out_chunk - b.first_chunk) << FDT_CHUNK_LG_SZ;
    const uint32_t cap = t->cap_of[payload_sz];                  /* payload_sz <= FDT_TPU_MTU: during_frag */
    const uint32_t li = (uint32_t)t->cur_in;
    if (!(b.link_mask >> li & 1u)) {
      b.link_mask |= 1u << li;
      b.link_first[li] = seq;
      b.guard_cur[li] = (uint32_t)b.cnt;
    }
    b.link_last[li] = seq;
    /* the frag's record is what the verifier reads: the device re-reads the
       frag's in-mcache line after the payload (link li + 1, seq) */
    fdgpu_frag_io_t &f = b.fio[b.cnt];          /* in place: no temporary (a wide reload of narrow stores stalls) */
    f.src = t->cur_src;
    f.sz = (uint32_t)payload_sz;
    f.out_off = (uint32_t)off;
    f.out_cap = cap;
    f.link = li + 1u;
    f.seq = seq;
    b.tso[b.cnt] = (uint32_t)*opt_tsorig;
    b.cnt++;
    b.end_off = off + cap;
    b.sig_cnt += fdt_frag_sig_bound(payload_sz);       /* (stats.sigs stays 0: the tile never sees the count) */
    t->out_chunk = fdt_dcache_compact_next(t->out_chunk, cap, t->cfg.out_chunk0, t->cfg.out_wmark);
    t->room_ok = false;
    /* the lap guard's span: the batch holds at most lap_span_max seqs of a
       link (this tile's next frag of the link is round_robin_cnt seqs on) */
    if (t->out_chunk <= b.first_chunk || b.cnt >= t->cfg.batch_txn_max ||
        b.sig_cnt + 16 > t->cfg.batch_sig_max || b.end_off + FRAG_CHUNKS * FDT_CHUNK_SZ > t->cfg.batch_bytes_max ||
        seq - b.link_first[li] + t->cfg.round_robin_cnt >= t->lap_span_max)
      b.closed = true;
    return;
  }
  if (t->gpu_parse) {
    /* the GPU parses: reserve the trailer the parse will produce (the
       payload's counts, fdt_txn_peek) and hand the payload over as a frag */
    (void)txn;
    const uint64_t sc = t->cur_sc, fp = t->cur_fp;
    VBatch &b = *t->open;
    if (!b.cnt) { b.first_chunk = t->out_chunk; b.t_first = now_ns(); b.cu_first = t->caught_up_cnt; }
    const uint64_t off = (t->out_chunk - b.first_chunk) << FDT_CHUNK_LG_SZ;
    __builtin_prefetch(b.items.data() + b.items.size() + 6, 1);      /* reserved: stores a few frags ahead */
    __builtin_prefetch(b.frags.data() + b.frags.size() + 12, 1);
    b.frags.push_back(fdgpu_frag_ex_t{(uint32_t)off, (uint32_t)payload_sz, (uint32_t)b.tr_used, (uint32_t)fp});
    b.items.push_back(VItem{seq, t->cur_tag, (uint32_t)t->out_chunk, (uint32_t)payload_sz, 1u, (uint32_t)*opt_tsorig,
                            (uint32_t)b.tr_used, (uint32_t)fp});
    b.cnt++;
    b.tr_used += (fp + 3) & ~3ull;
    b.end_off = off + payload_sz;
    b.sig_cnt += fdt_frag_sig_bound(payload_sz);
    if (sc >= 1 && sc <= 16) t->st.sigs += sc;
    t->out_chunk = fdt_dcache_compact_next(t->out_chunk, toff + fp + 2, t->cfg.out_chunk0, t->cfg.out_wmark);
    t->room_ok = false;
    if (t->out_chunk <= b.first_chunk || b.cnt >= t->cfg.batch_txn_max ||
        b.sig_cnt + 16 > t->cfg.batch_sig_max || b.end_off + FRAG_CHUNKS * FDT_CHUNK_SZ > t->cfg.batch_bytes_max)
      b.closed = true;
    return;
  }
  uint8_t *txn_t = txn + toff;
  if (toff != payload_sz) txn[payload_sz] = 0;
  const uint64_t tsz = fdt_txn_parse(txn, payload_sz, txn_t, nullptr);
  if (!tsz) {                                           /* fd_verify.c:117-121 */
    t->st.parse_fail++;
    t->log(seq, FDGPU_VTILE_LOG_PARSE_FAIL);
    *opt_filter = 1;
    return;
  }
  const uint16_t psz = (uint16_t)payload_sz;
  std::memcpy(txn_t + tsz, &psz, 2);
  const uint64_t new_sz = toff + tsz + 2;
  const fdt_txn_t *tt = (const fdt_txn_t *)txn_t;
  VBatch &b = *t->open;                                 /* after_credit made sure one is open */
  if (!b.cnt) { b.first_chunk = t->out_chunk; b.t_first = now_ns(); b.cu_first = t->caught_up_cnt; }
  const uint64_t off = (t->out_chunk - b.first_chunk) << FDT_CHUNK_LG_SZ;
  fdgpu_txn_t d;
  d.msg_off = (uint32_t)(off + tt->message_off);
  d.msg_sz = (uint32_t)(payload_sz - tt->message_off);
  d.sig_off = (uint32_t)(off + tt->signature_off);
  d.pub_off = (uint32_t)(off + tt->acct_addr_off);
  d.sig_cnt = tt->signature_cnt;
  b.txns.push_back(d);
  b.items.push_back(VItem{seq, fdt_hash(t->cfg.hashmap_seed, txn + tt->signature_off, 64), (uint32_t)t->out_chunk,
                          (uint32_t)new_sz, tt->signature_off, (uint32_t)*opt_tsorig, 0u, 0u});
  b.cnt++;
  b.end_off = off + new_sz;
  if (tt->signature_cnt <= 16) { b.sig_cnt += tt->signature_cnt; t->st.sigs += tt->signature_cnt; }
  t->out_chunk = fdt_dcache_compact_next(t->out_chunk, new_sz, t->cfg.out_chunk0, t->cfg.out_wmark);
  t->room_ok = false;
  /* the arena must stay one contiguous run of chunks: a wrapped cursor closes it */
  if (t->out_chunk <= b.first_chunk || b.cnt >= t->cfg.batch_txn_max ||
      b.sig_cnt + 16 > t->cfg.batch_sig_max || b.end_off + FRAG_CHUNKS * FDT_CHUNK_SZ > t->cfg.batch_bytes_max)
    b.closed = true;
  /* accepted: published later, in order, by after_credit (MANUAL_PUBLISH) */
}

/* after_credit runs once per mux loop iteration, i.e. about once per frag:
   the verifier is polled (an event query) and the partial-batch timer read
   only every 64th call, or at once when the tile cannot take the next frag
   or is mid-way through publishing a completed batch. */
__attribute__((always_inline)) inline void vm_after_credit(void *ctx, fdt_mux_context_t *mux, int *opt_poll_in) {
  auto *t = (fdgpu_vmux *)ctx;
  if (t->error) { *opt_poll_in = 0; return; }
  const bool due = (++t->calls & 63u) == 0;
  if (due) {                                   /* the tile's longest stall between two of these */
    const uint64_t now = __rdtsc();
    if (t->due_tsc) t->stall_max_tick = std::max(t->stall_max_tick, now - t->due_tsc);
    t->due_tsc = now;
  }
  const bool stuck = t->open ? t->open->closed : t->pool.empty();
  if (due || stuck || (!t->inflight.empty() && t->inflight.front()->done)) t->resolve(mux, opt_poll_in);
  if (due || stuck) t->submit();
  if (!*opt_poll_in || t->error || !t->can_take()) { *opt_poll_in = 0; return; }
  if (!t->room_ok && !(t->room_ok = t->room(mux))) { *opt_poll_in = 0; t->st.backpressure++; }
}

/* ... or straight into the verify tile's callbacks, inlined into its own
   instance of the loop, with the round-robin filter applied as a skip */
struct VmHooks {
  fdgpu_vmux *t;
  void metrics_write() {}
  void during_housekeeping() {}
  void before_credit(fdt_mux_context_t *) {}
  void after_credit(fdt_mux_context_t *m, int *p) { vm_after_credit(t, m, p); }
  /* seqs of link i from seq on that another tile of the round robin takes */
  uint64_t skip(uint64_t, uint64_t seq) const {
    const uint64_t cnt = t->cfg.round_robin_cnt;
    if (cnt == 1) return 0;
    const uint64_t r = t->rr_mask ? (seq & t->rr_mask) : seq % cnt, idx = t->cfg.round_robin_idx;
    return idx >= r ? idx - r : idx + cnt - r;
  }
  void caught_up(uint64_t) { t->caught_up_cnt++; }
  void skipped(uint64_t, uint64_t seq, uint64_t k) {
    t->st.in_frags += k;
    t->st.filtered_rr += k;
    for (uint64_t j = 0; j < k; j++) t->log(seq + j, FDGPU_VTILE_LOG_FILTERED);
  }
  bool has_before_frag() const { return true; }
  void before_frag(uint64_t i, uint64_t seq, uint64_t sig, int *f) { vm_before_frag(t, i, seq, sig, f); }
  void during_frag(uint64_t i, uint64_t seq, uint64_t sig, uint64_t chunk, uint64_t sz, int *f) {
    vm_during_frag(t, i, seq, sig, chunk, sz, f);
  }
  void after_frag(uint64_t i, uint64_t seq, uint64_t *sig, uint64_t *chunk, uint64_t *sz, uint64_t *tsorig, int *f,
                  fdt_mux_context_t *m) {
    vm_after_frag(t, i, seq, sig, chunk, sz, tsorig, f, m);
  }
};

bool is_vmux_callbacks(const fdt_mux_callbacks_t *cb) {
  return cb->before_frag == vm_before_frag && cb->during_frag == vm_during_frag && cb->after_frag == vm_after_frag &&
         cb->after_credit == vm_after_credit && !cb->before_credit && !cb->during_housekeeping && !cb->metrics_write;
}

int vmux_loop(const fdt_mux_cfg_t *cfg, void *ctx, const volatile uint64_t *halt, fdt_mux_stats_t *stats_out) {
  VmHooks h{(fdgpu_vmux *)ctx};
  h.t->sees_caught_up = true;
  const int rc = mux_loop(cfg, h, halt, stats_out);
  h.t->sees_caught_up = false;
  return rc;
}

}  // namespace

extern "C" {

uint64_t fdgpu_vmux_dcache_data_sz(uint64_t cr_max, uint32_t batch_txn_max, uint32_t inflight_max) {
  if (!inflight_max) inflight_max = 2;
  return (cr_max + (2 * (uint64_t)inflight_max + 1) * batch_txn_max + 2) * FRAG_CHUNKS * FDT_CHUNK_SZ;
}

fdgpu_vmux_t *fdgpu_vmux_new(const fdgpu_vmux_cfg_t *cfg, fdgpu_verifier_t ver) {
  if (!cfg || !ver.submit || !ver.poll || !cfg->out_base || !cfg->batch_txn_max || !cfg->cr_max ||
      cfg->in_cnt > FDT_MUX_IN_MAX || cfg->out_wmark < cfg->out_chunk0)
    return nullptr;
  for (uint64_t i = 0; i < cfg->in_cnt; i++) if (!cfg->in_base[i]) return nullptr;
  auto *t = new (std::nothrow) fdgpu_vmux;
  if (!t) return nullptr;
  t->cfg = *cfg;
  fdgpu_vmux_cfg_t &c = t->cfg;
  t->gpu_parse = cfg->gpu_parse != 0;
  t->gather = cfg->gpu_parse == 2;
  if (cfg->gpu_parse > 2 || (t->gpu_parse && !t->gather && (!ver.submit_frags || !ver.poll_frags)) ||
      (t->gather && (!ver.submit_io || !ver.poll_io))) {
    delete t;
    return nullptr;
  }
  if (t->gather) {
    /* an unlapped line must mean an intact payload: each in dcache holds
       depth + 1 maximal frags (fdt_dcache_data_sz), or is a TPU reassembly
       slot arena of depth + burst slots (the same span from chunk0 to wmark) */
    const uint64_t mtu_chunks = ((FDT_TPU_MTU + 2 * FDT_CHUNK_SZ - 1) >> (1 + FDT_CHUNK_LG_SZ)) << 1;
    for (uint64_t i = 0; i < cfg->in_cnt; i++)
      if (!cfg->in_mcache[i] || !pow2(cfg->in_depth[i]) || cfg->in_wmark[i] < cfg->in_chunk0[i] ||
          cfg->in_wmark[i] - cfg->in_chunk0[i] < cfg->in_depth[i] * mtu_chunks) {
        delete t;
        return nullptr;
      }
    uint64_t dmin = UINT64_MAX;
    for (uint64_t i = 0; i < cfg->in_cnt; i++) {
      t->links[i] = fdgpu_link_t{(uint64_t)(uintptr_t)cfg->in_mcache[i], cfg->in_depth[i]};
      dmin = std::min(dmin, cfg->in_depth[i]);
    }
    t->lap_span_max = cfg->lap_span_max ? cfg->lap_span_max : std::max<uint64_t>(dmin / 2, 1);
    t->lap_margin = cfg->lap_margin ? cfg->lap_margin : std::max<uint64_t>(dmin / 4, 1);
  }
  if (!c.round_robin_cnt) c.round_robin_cnt = 1;
  if (!c.inflight_max) c.inflight_max = 2;
  if (!c.tcache_depth) c.tcache_depth = FDT_VERIFY_TCACHE_DEPTH;
  if (!cfg->tcache_depth && !c.tcache_map_cnt) c.tcache_map_cnt = FDT_VERIFY_TCACHE_MAP_CNT;
  if (!c.batch_sig_max) c.batch_sig_max = std::max<uint64_t>(16, (uint64_t)c.batch_txn_max * 12);
  if (!c.batch_bytes_max) c.batch_bytes_max = (uint64_t)c.batch_txn_max * FRAG_CHUNKS * FDT_CHUNK_SZ;
  /* the ring must hold two maximal frags; a batch one */
  if (c.batch_sig_max < 16 || c.batch_bytes_max < FRAG_CHUNKS * FDT_CHUNK_SZ ||
      c.out_wmark - c.out_chunk0 < 2 * FRAG_CHUNKS) {
    delete t;
    return nullptr;
  }
  const uint64_t fp = fdt_tcache_footprint(c.tcache_depth, c.tcache_map_cnt);
  if (!fp) { delete t; return nullptr; }
  t->tcache_mem.assign(fp / 8, 0);
  t->tcache = fdt_tcache_new(t->tcache_mem.data(), c.tcache_depth, c.tcache_map_cnt);
  t->use_ring = c.tcache_depth <= FDT_TAGRING_MAX;
  if (t->gather) {
    t->cap_of.resize(FDT_TPU_MTU + 1);
    for (uint64_t sz = 0; sz <= FDT_TPU_MTU; sz++) t->cap_of[sz] = (uint16_t)(align2(sz) + fdt_frag_fp_bound(sz) + 2);
  }
  fdt_tagring_init(&t->ring, c.tcache_depth);
  t->ver = ver;
  t->st.lap_margin_min = UINT64_MAX;
  t->out_chunk = c.out_chunk0;
  t->rr_mask = (c.round_robin_cnt & (c.round_robin_cnt - 1)) == 0 ? c.round_robin_cnt - 1 : 0;
  uint64_t n = 1;
  while (n < c.cr_max) n <<= 1;
  t->pub_chunk.assign(n, 0);
  t->pub_mask = n - 1;
  t->storage.resize(2 * (uint64_t)c.inflight_max + 1);    /* on the GPU, done but not yet published, open */
  for (auto &b : t->storage) {
    b.codes.resize(c.batch_txn_max);
    b.txns.reserve(c.batch_txn_max);
    if (t->gpu_parse && !t->gather) b.frags.reserve(c.batch_txn_max);
    if (t->gather) {
      b.fio.resize(c.batch_txn_max); b.tso.resize(c.batch_txn_max);
      b.tags.resize(c.batch_txn_max); b.out_szs.resize(c.batch_txn_max);
    } else {
      b.items.reserve(c.batch_txn_max);
    }
    t->pool.push_back(&b);
  }
  return t;
}

void fdgpu_vmux_delete(fdgpu_vmux_t *t) {
  if (!t) return;
  for (VBatch *b : t->inflight)                 /* the verifier may still write codes / read the arena */
    if (!b->done) {
      if (t->gather) t->ver.poll_io(t->ver.ctx, b->ticket, b->codes.data(), b->tags.data(), b->out_szs.data(), 1);
      else if (t->gpu_parse) t->ver.poll_frags(t->ver.ctx, b->ticket, b->codes.data(), b->trailers.data(), 1);
      else t->ver.poll(t->ver.ctx, b->ticket, b->codes.data(), 1);
    }
  delete t;
}

fdt_mux_callbacks_t fdgpu_vmux_callbacks(void) {
  fdt_mux_callbacks_t cb{};
  cb.before_frag = vm_before_frag;
  cb.during_frag = vm_during_frag;
  cb.after_frag = vm_after_frag;
  cb.after_credit = vm_after_credit;
  return cb;
}

void fdgpu_vmux_stats(const fdgpu_vmux_t *t, fdgpu_vtile_stats_t *out) {
  *out = t->st;
  out->stall_max_ns = (uint64_t)((double)t->stall_max_tick / tick_per_ns());
  out->lat_cnt = t->lat.size();
}

int fdgpu_vmux_idle(const fdgpu_vmux_t *t) {
  return t->inflight.empty() && (!t->open || !t->open->cnt);
}

int fdgpu_vmux_error(const fdgpu_vmux_t *t) { return t->error; }

uint64_t fdgpu_vmux_final_cnt(const fdgpu_vmux_t *t) { return t->final_cnt.load(std::memory_order_acquire); }

uint64_t fdgpu_vmux_latencies(const fdgpu_vmux_t *t, uint64_t *out, uint64_t max) {
  const uint64_t n = std::min<uint64_t>(max, t->lat.size());
  std::memcpy(out, t->lat.data(), n * 8);
  return n;
}

void fdgpu_vmux_log_enable(fdgpu_vmux_t *t, uint64_t log_max) {
  t->log_max = log_max;
  t->log_seq.reserve(log_max);
  t->log_code.reserve(log_max);
}

uint64_t fdgpu_vmux_log(const fdgpu_vmux_t *t, uint64_t *seqs, int8_t *codes, uint64_t max) {
  const uint64_t n = std::min<uint64_t>(max, t->log_seq.size());
  std::memcpy(seqs, t->log_seq.data(), n * 8);
  std::memcpy(codes, t->log_code.data(), n);
  return n;
}

}  // extern "C"
