/* fdgpu_engine.cpp -- host side of the MI355X Ed25519 verify engine and the
   exported C ABI (include/fd_ed25519_gpu.h).

   Per engine (one per GPU):
     - `ring_depth` staging slots, each with pinned host buffers, device
       buffers, its own stream and its own workspace: a slot's H2D copy,
       verify kernels and D2H of the codes run in order on its stream, and
       the slots' batches overlap each other on the GPU (copies of one batch
       under the kernels of another; two small batches sharing the CUs);
     - one compute stream + workspace for the device-resident path
       (fdgpu_dev_batch_*, fdgpu_verify_device) and the diagnostics;
     - the fixed-base comb table (built on the device at open).
   Untrusted descriptors are bounds-checked on the host before anything is
   handed to the GPU (offsets + sizes must lie inside the arena). */
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fd_ed25519_gpu.h"
#include "fdgpu_internal.h"
#include "fdt_parse.h"

#define FDT_TXN_MAX_SZ_BYTES 852u   /* FD_TXN_MAX_SZ (fd_txn.h:98): one parsed fd_txn_t record */
#define FDT_TXN_MTU_BYTES 1232u     /* FD_TXN_MTU (fd_txn.h:103) */

namespace {

thread_local std::string g_err;

void set_err(const char *fmt, ...) {
  char buf[512];
  va_list ap; va_start(ap, fmt); vsnprintf(buf, sizeof buf, fmt, ap); va_end(ap);
  g_err = buf;
}

#define HIPCHK(x, ret) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  set_err("%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); return ret; } } while (0)

}  // namespace

/* FDGPU_SUBMIT_PROF=1: where fdgpu_submit_frags_io's time goes (validation
   loop, enqueue of copies and kernels), printed at engine close */
namespace {
std::atomic<uint64_t> g_sp_loop{0}, g_sp_enq{0}, g_sp_calls{0}, g_sp_frags{0};
inline uint64_t sp_now() { timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts); return ts.tv_sec * 1000000000ull + ts.tv_nsec; }
const bool g_sp_on = getenv("FDGPU_SUBMIT_PROF") && getenv("FDGPU_SUBMIT_PROF")[0] == '1';
/* FDGPU_IO_DMA=1: gathered batches read their payloads by DMA, the source
   ranges copied into a device mirror and parsed there (engine alone, two
   engines: 86-89 vs 80-81 M txn/s); default off, the ingest kernel's loads over
   the bus: in the mux tiles the ranges of two tiles sharing a link interleave
   (each copy carries the other tile's payloads too) and the range building
   sits on the tile's thread -- two tiles 42-59 M with DMA vs 71-72 M
   without (profiles/r05/aux_blocks.md) */
const bool g_io_dma = getenv("FDGPU_IO_DMA") && getenv("FDGPU_IO_DMA")[0] == '1';
/* FDGPU_BIG_STREAMS=0: big ring batches verify on their own slot streams (A/B) */
const bool g_big_off = getenv("FDGPU_BIG_STREAMS") && getenv("FDGPU_BIG_STREAMS")[0] == '0';
/* the last FDGPU_ST_RING fdgpu_submit calls of the process: {staging copy,
   descriptor expansion, enqueue} ns (fdgpu_debug_submit_times).  Each call
   writes the entry its fetch_add drew; the words are relaxed atomics, so
   concurrent submitters and a reader never race (a reader may see a triple
   that a writer is mid-way through, which is a diagnostic's tolerance) */
constexpr uint64_t FDGPU_ST_RING = 8192;
std::atomic<uint64_t> g_st[FDGPU_ST_RING][3];
std::atomic<uint64_t> g_st_n{0};
}

namespace {

struct Slot {
  hipStream_t stream = nullptr;
  hipEvent_t h2d_done = nullptr, comp_done = nullptr, done = nullptr;
  uint8_t *h_arena = nullptr, *d_arena = nullptr;
  fdgpu_sig_desc_t *h_sigs = nullptr, *d_sigs = nullptr;
  uint32_t *h_perm = nullptr, *d_perm = nullptr;   /* block-count grouping: descriptor i -> signature perm[i] */
  fdgpu_txn_desc_t *h_txns = nullptr, *d_txns = nullptr;
  int8_t *h_codes = nullptr, *d_txn_codes = nullptr, *d_sig_codes = nullptr;
  uint32_t *d_ws = nullptr;   /* this slot's workspace: slots run concurrently on their own streams; */
  uint64_t ws_sig = 0;        /* sized on demand to the largest batch the slot has carried */
  int64_t ticket = -1;      /* -1: free */
  uint64_t k_sigs = 0;      /* signatures (the launch's bound) of its verify: FDGPU_FLAG_PAIR_AUTO's load */
  uint64_t k_lanes = 0;     /* and its lanes (two per signature for the two-lane kernel): FDGPU_FLAG_SPREAD_AUTO's */
  bool staged = false;      /* reserved by fdgpu_stage_acquire, not yet submitted */
  bool held = false;        /* polled with fdgpu_poll_keep, awaiting fdgpu_release */
  uint64_t txn_cnt = 0;
  /* completion word in pinned host memory: the slot's stream writes
     flag_seq into it after the code read-back (hipStreamWriteValue32), so a
     non-blocking poll is one host load instead of a runtime event query */
  uint32_t *h_flag = nullptr, *d_flag = nullptr;
  uint32_t flag_seq = 0;
  uint32_t polls = 0;         /* non-blocking polls of the current batch (stream error checks) */
  uint64_t last_query = 0;    /* when a poll last asked the runtime (ns) */
  /* frag batches (fdgpu_submit_frags): GPU-side parse buffers, allocated on
     the slot's first frag batch; the trailer buffers grow to the batches */
  bool frag = false;          /* the batch in flight is a frag batch */
  fdgpu_frag_ex_t *h_fx = nullptr, *d_fx = nullptr;
  uint8_t *d_txn_out = nullptr;
  uint16_t *d_txn_sz = nullptr;
  fdgpu_txn_t *d_txd = nullptr;
  uint32_t *d_cnt = nullptr, *d_sig0 = nullptr, *d_blocktot = nullptr, *d_n_sig = nullptr;
  uint8_t *d_tr = nullptr, *h_tr = nullptr;   /* [codes, padded to 64][trailers]: one read-back */
  uint64_t tr_cap = 0, tr_sz = 0, tr_base = 0;
  /* gathered frag batches (fdgpu_submit_frags_io): the payloads' device-side
     addresses, and the out image the finish kernel assembles (grown on
     demand); the read-back is [codes][tags][out sizes] in h_tr */
  bool io = false;
  uint8_t *h_io = nullptr, *d_ioh = nullptr;  /* pinned [frag records][payload addresses]; its device view */
  fdgpu_frag_ex_t *d_fxio = nullptr;          /* the records, kept on the device by the ingest */
  uint32_t *d_io_cnt = nullptr;               /* the ingest's signature count: zero at the start of a gathered
                                                 batch (cleared by the finish of the slot's previous one) */
  bool io_cnt_dirty = false;                  /* an ingest was queued but not its finish (an error between
                                                 them): the next gathered batch clears the count first */
  uint8_t *d_mirror = nullptr;                /* DMA gather: the batch's source ranges, copied in by the DMA
                                                 engines, parsed and verified in place (the batch arena) */
  uint64_t mirror_cap = 0;
  uint8_t *d_trh = nullptr;                   /* h_tr's device-side address (results written in place) */
  /* FDGPU_FLAG_MERGE: the batch's gather + parse are queued and its verify
     waits to be merged with the other batches ready (merge_kick), which then
     queues the rest of the batch behind it */
  hipEvent_t parsed = nullptr;
  bool vpending = false;
  bool failed = false;        /* its merged verify could not be queued: the next poll reports the error */
  uint32_t m_n = 0;
  uint64_t m_seed = 0, m_cb = 0, m_bound = 0;
  uint8_t *m_out = nullptr;
  uint8_t *m_arena = nullptr;   /* the batch arena (d_arena, or d_mirror for a DMA-gathered batch) */
};

/* poll_slot answers a pending batch without the ring lock, reading a slot's
   ticket, held, flag_seq and polls atomically; every write of those fields
   (under ring_mu) is an atomic store too, so the two sides never race */
template <class T> inline void st_rlx(T &f, T v) { __atomic_store_n(&f, v, __ATOMIC_RELAXED); }
inline void slot_flag_next(Slot *s) { __atomic_store_n(&s->flag_seq, s->flag_seq + 1, __ATOMIC_RELEASE); }

/* a merge stream of an FDGPU_FLAG_MERGE engine */
struct Merge {
  hipStream_t stream = nullptr;
  uint32_t *h_flag = nullptr, *d_flag = nullptr;   /* seq after each merged verify: free when equal */
  uint32_t seq = 0;
  fdgpu_mbatch_t *h_tab = nullptr, *d_tab = nullptr;   /* tabs x ring_depth batch entries, pinned */
  std::vector<hipEvent_t> ev;                          /* one per table: the launch that read it is done */
};

}  // namespace

struct fdgpu_engine {
  int device = 0;
  fdgpu_cfg_t cfg{};
  hipStream_t compute = nullptr;
  uint32_t *d_btab = nullptr;
  uint32_t *d_ws = nullptr;          /* per-lane A-table workspace, fdgpu_ws_bytes(ws_sig) */
  size_t ws_bytes = 0;
  uint64_t ws_sig = 0;
  uint32_t resident_blocks = 0;     /* verify-kernel occupancy x CUs (fallback grid cap, reporting) */
  uint64_t kc_seed = 0;             /* key cache hash seed, drawn at open */
  std::vector<Slot> slots;
  int64_t next_ticket = 0;
  int8_t *d_scratch_codes = nullptr;   /* for fdgpu_verify_device with d_sig_codes == NULL */
  uint64_t scratch_cap = 0;
  std::vector<hipStream_t> batch_streams;   /* streams of device batches with their own queue */
  /* ring batches that fill the chip on their own (FDGPU_BIG_SIGS) verify on
     these two streams in turn, not on their slot's: see submit_slot */
  hipStream_t big[2] = {nullptr, nullptr};
  uint32_t big_rr = 0;
  /* the ring API (submit / stage / poll / release) may be called from several
     host threads (verify tiles sharing the node's engines) */
  std::mutex ring_mu;
  bool flag_poll = false;            /* slots signal completion through h_flag (probed at open) */
  /* fdgpu_host_register calls of this engine, one entry each (a range
     registered twice holds two references): the page-aligned start the
     caller named, and the pinned region [base, end) that covers it */
  struct Reg { uintptr_t user, base, end, dbase; };   /* dbase: the region's device-side address */
  std::vector<Reg> regions;
  bool drop_flag = false;            /* test hook (FDGPU_DEBUG_DROP_FLAG=1): the stream never writes the
                                        completion word, so polls must finish through the event */
  uint32_t fail_merge_at = 0;        /* test hook (FDGPU_DEBUG_FAIL_MERGE=k): the k-th merge launch fails
                                        before queueing anything, as a HIP error part-way would */
  uint32_t merge_calls = 0;
  /* FDGPU_FLAG_MERGE */
  std::vector<Merge> merges;
  std::vector<Slot *> pending;       /* batches parsed (or parsing) whose verify is not launched */
  uint32_t merge_rr = 0, merge_tabs = 0;
  uint64_t merge_launches = 0, merge_batches = 0;
};

namespace {

void slot_free(Slot &s) {
  if (s.stream) (void)hipStreamDestroy(s.stream);
  if (s.h2d_done) (void)hipEventDestroy(s.h2d_done);
  if (s.comp_done) (void)hipEventDestroy(s.comp_done);
  if (s.done) (void)hipEventDestroy(s.done);
  if (s.parsed) (void)hipEventDestroy(s.parsed);
  if (s.h_arena) (void)hipHostFree(s.h_arena);
  if (s.h_sigs) (void)hipHostFree(s.h_sigs);
  if (s.h_perm) (void)hipHostFree(s.h_perm);
  if (s.d_perm) (void)hipFree(s.d_perm);
  if (s.h_txns) (void)hipHostFree(s.h_txns);
  if (s.h_codes) (void)hipHostFree(s.h_codes);
  if (s.d_arena) (void)hipFree(s.d_arena);
  if (s.d_sigs) (void)hipFree(s.d_sigs);
  if (s.d_txns) (void)hipFree(s.d_txns);
  if (s.d_txn_codes) (void)hipFree(s.d_txn_codes);
  if (s.d_sig_codes) (void)hipFree(s.d_sig_codes);
  if (s.d_ws) (void)hipFree(s.d_ws);
  if (s.h_flag) (void)hipHostFree(s.h_flag);
  if (s.h_fx) (void)hipHostFree(s.h_fx);
  if (s.h_tr) (void)hipHostFree(s.h_tr);
  if (s.h_io) (void)hipHostFree(s.h_io);
  for (void *p : {(void *)s.d_fx, (void *)s.d_txn_out, (void *)s.d_txn_sz, (void *)s.d_txd, (void *)s.d_cnt,
                  (void *)s.d_sig0, (void *)s.d_blocktot, (void *)s.d_n_sig, (void *)s.d_tr, (void *)s.d_fxio,
                  (void *)s.d_io_cnt, (void *)s.d_mirror})
    if (p) (void)hipFree(p);
  s = Slot{};
}

bool slot_alloc(Slot &s, const fdgpu_cfg_t &c) {
  const size_t arena = c.max_arena + FDGPU_ARENA_SLACK;
  HIPCHK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking), false);
  HIPCHK(hipEventCreateWithFlags(&s.h2d_done, hipEventDisableTiming), false);
  HIPCHK(hipEventCreateWithFlags(&s.comp_done, hipEventDisableTiming), false);
  HIPCHK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming), false);
  HIPCHK(hipEventCreateWithFlags(&s.parsed, hipEventDisableTiming), false);
  HIPCHK(hipHostMalloc((void **)&s.h_arena, arena, hipHostMallocDefault), false);
  HIPCHK(hipHostMalloc((void **)&s.h_sigs, c.max_sig * sizeof(fdgpu_sig_desc_t) + 16, hipHostMallocDefault), false);
  HIPCHK(hipHostMalloc((void **)&s.h_perm, c.max_sig * sizeof(uint32_t) + 16, hipHostMallocDefault), false);
  HIPCHK(hipHostMalloc((void **)&s.h_txns, c.max_txn * sizeof(fdgpu_txn_desc_t) + 16, hipHostMallocDefault), false);
  HIPCHK(hipHostMalloc((void **)&s.h_codes, c.max_txn + 16, hipHostMallocDefault), false);
  HIPCHK(hipMalloc((void **)&s.d_arena, arena), false);
  HIPCHK(hipMalloc((void **)&s.d_sigs, c.max_sig * sizeof(fdgpu_sig_desc_t) + 16), false);
  HIPCHK(hipMalloc((void **)&s.d_perm, c.max_sig * sizeof(uint32_t) + 16), false);
  HIPCHK(hipMalloc((void **)&s.d_txns, c.max_txn * sizeof(fdgpu_txn_desc_t) + 16), false);
  HIPCHK(hipMalloc((void **)&s.d_txn_codes, c.max_txn + 16), false);
  HIPCHK(hipMalloc((void **)&s.d_sig_codes, c.max_sig + 16), false);
  HIPCHK(hipHostMalloc((void **)&s.h_flag, 64, hipHostMallocDefault), false);   /* own cache line */
  *s.h_flag = 0;
  HIPCHK(hipHostGetDevicePointer((void **)&s.d_flag, s.h_flag, 0), false);
  return true;
}

/* Grow the slot's workspace to cover n_sig signatures (the slot is free, so
   nothing of its stream still reads the old one).  Grown by half again each
   time, so a default engine (65,536 txns, up to 12 signatures each) holds
   what its batches actually carry, not 12 x 3.2 KB per txn up front. */
bool slot_ws(Slot &s, uint64_t n_sig) {
  if (s.d_ws && n_sig <= s.ws_sig) return true;
  const uint64_t want = std::max<uint64_t>(n_sig, s.ws_sig + s.ws_sig / 2);
  if (s.d_ws) { HIPCHK(hipStreamSynchronize(s.stream), false); (void)hipFree(s.d_ws); s.d_ws = nullptr; s.ws_sig = 0; }
  if (hipMalloc((void **)&s.d_ws, fdgpu_ws_bytes(want ? want : 1)) != hipSuccess) {
    if (want == n_sig || hipMalloc((void **)&s.d_ws, fdgpu_ws_bytes(n_sig ? n_sig : 1)) != hipSuccess) {
      (void)hipGetLastError();
      s.d_ws = nullptr;
      set_err("slot workspace alloc (%llu signatures)", (unsigned long long)n_sig);
      return false;
    }
    s.ws_sig = n_sig ? n_sig : 1;
    return true;
  }
  s.ws_sig = want ? want : 1;
  return true;
}

/* The slot's GPU-side parse buffers (first frag batch) and a trailer
   buffer of at least tr bytes (the slot is free: nothing reads them). */
bool slot_frag_bufs(Slot &s, const fdgpu_cfg_t &c, uint64_t tr) {
  if (!s.d_fx) {
    const uint64_t n = c.max_txn + 1, nb = (c.max_txn + 1023) / 1024 + 2;
    HIPCHK(hipHostMalloc((void **)&s.h_fx, n * sizeof(fdgpu_frag_ex_t), hipHostMallocDefault), false);
    HIPCHK(hipMalloc((void **)&s.d_fx, n * sizeof(fdgpu_frag_ex_t)), false);
    HIPCHK(hipMalloc((void **)&s.d_txn_out, n * FDT_TXN_MAX_SZ_BYTES), false);
    HIPCHK(hipMalloc((void **)&s.d_txn_sz, n * sizeof(uint16_t)), false);
    HIPCHK(hipMalloc((void **)&s.d_txd, n * sizeof(fdgpu_txn_t)), false);
    HIPCHK(hipMalloc((void **)&s.d_cnt, n * sizeof(uint32_t)), false);
    HIPCHK(hipMalloc((void **)&s.d_sig0, n * sizeof(uint32_t)), false);
    HIPCHK(hipMalloc((void **)&s.d_blocktot, nb * sizeof(uint32_t)), false);
    HIPCHK(hipMalloc((void **)&s.d_n_sig, sizeof(uint32_t)), false);
  }
  tr += (c.max_txn + 64) & ~63ull;                      /* the codes go in front of the trailers */
  if (tr > s.tr_cap) {
    HIPCHK(hipStreamSynchronize(s.stream), false);
    if (s.d_tr) { (void)hipFree(s.d_tr); s.d_tr = nullptr; }
    if (s.h_tr) { (void)hipHostFree(s.h_tr); s.h_tr = nullptr; }
    s.tr_cap = 0;
    const uint64_t want = std::max<uint64_t>(tr + tr / 4, 256 * 1024);
    HIPCHK(hipMalloc((void **)&s.d_tr, want), false);
    HIPCHK(hipHostMalloc((void **)&s.h_tr, want, hipHostMallocDefault), false);
    HIPCHK(hipHostGetDevicePointer((void **)&s.d_trh, s.h_tr, 0), false);
    s.tr_cap = want;
  }
  return true;
}

/* The slot's gathered-batch buffers (fdgpu_submit_frags_io), on first use:
   pinned [frag records][payload addresses][re-check pairs] the gather reads
   in place, and the records' device copy. */
/* DMA gather: the batch's ranges may also carry other tiles' frags lying
   between this batch's (a round robin of two takes every other frag of a
   link), so the mirror holds twice the engine's arena */
inline uint64_t mirror_bytes(const fdgpu_cfg_t &c) { return 2 * c.max_arena + FDGPU_ARENA_SLACK + 4096; }

bool slot_io_bufs(Slot &s, const fdgpu_cfg_t &c) {
  if (s.h_io) return true;
  const uint64_t m = c.max_txn + 1,
                 bytes = m * (sizeof(fdgpu_frag_ex_t) + 3 * sizeof(uint64_t)) + 192 + FDGPU_IO_RANGES_MAX * 8;
  HIPCHK(hipHostMalloc((void **)&s.h_io, bytes, hipHostMallocDefault), false);
  HIPCHK(hipHostGetDevicePointer((void **)&s.d_ioh, s.h_io, 0), false);
  HIPCHK(hipMalloc((void **)&s.d_fxio, m * sizeof(fdgpu_frag_ex_t)), false);
  HIPCHK(hipMalloc((void **)&s.d_io_cnt, 64), false);
  if (g_io_dma) {
    HIPCHK(hipMalloc((void **)&s.d_mirror, mirror_bytes(c)), false);
    s.mirror_cap = mirror_bytes(c) - FDGPU_ARENA_SLACK - 4096;
  }
  HIPCHK(hipMemsetAsync(s.d_io_cnt, 0, 64, s.stream), false);    /* ordered before the slot's first batch */
  return true;
}

/* SHA-512 blocks of R || A || M (fdgpu_sha512.h sha512_hram_blocks) */
inline uint32_t hram_blocks(uint32_t msg_sz) { return (64u + msg_sz + 16u) / 128u + 1u; }

/* Validate and expand transactions into per-signature work items.
   Returns the number of signatures or -1 on invalid input.

   perm != NULL: the descriptors are grouped by SHA-512 block count (a
   stable counting sort; the SHA loop of a wave runs to its longest
   message, so mixed message sizes in one wave cost the longest one's
   blocks) and perm[i] is the signature index (in transaction order, the
   combine kernel's sig0 + j) of descriptor i.  perm == NULL: transaction
   order, no permutation. */
int64_t expand(uint64_t arena_sz, const fdgpu_txn_t *txns, uint64_t txn_cnt, uint64_t max_sig,
               fdgpu_sig_desc_t *sigs, fdgpu_txn_desc_t *tds, uint32_t *perm) {
  uint64_t ns = 0;
  uint64_t cnt_by_grp[FDGPU_NBLK_GROUPS] = {};
  for (uint64_t t = 0; t < txn_cnt; t++) {
    const fdgpu_txn_t &x = txns[t];
    const uint32_t cnt = x.sig_cnt;
    tds[t].sig0 = (uint32_t)ns;
    tds[t].sig_cnt = cnt;
    if (cnt == 0 || cnt > 16) { tds[t].sig_cnt = 0; continue; }   /* -> ERR_SIG without verifying */
    if ((uint64_t)x.msg_off + x.msg_sz > arena_sz || (uint64_t)x.sig_off + 64ull * cnt > arena_sz ||
        (uint64_t)x.pub_off + 32ull * cnt > arena_sz) {
      set_err("txn %llu: descriptor out of arena bounds", (unsigned long long)t);
      return -1;
    }
    if (ns + cnt > max_sig) { set_err("batch exceeds max_sig (%llu)", (unsigned long long)max_sig); return -1; }
    if (perm) cnt_by_grp[std::min(hram_blocks(x.msg_sz), FDGPU_NBLK_GROUPS) - 1] += cnt;
    ns += cnt;
  }
  uint64_t next[FDGPU_NBLK_GROUPS];
  if (perm) {
    uint64_t o = 0;
    for (uint32_t g = 0; g < FDGPU_NBLK_GROUPS; g++) { next[g] = o; o += cnt_by_grp[g]; }
  }
  for (uint64_t t = 0; t < txn_cnt; t++) {
    const fdgpu_txn_t &x = txns[t];
    const uint32_t cnt = tds[t].sig_cnt;
    if (!cnt) continue;
    const uint32_t s0 = tds[t].sig0;
    uint64_t *slot = perm ? &next[std::min(hram_blocks(x.msg_sz), FDGPU_NBLK_GROUPS) - 1] : nullptr;
    for (uint32_t j = 0; j < cnt; j++) {
      const uint64_t i = slot ? (*slot)++ : (uint64_t)s0 + j;
      sigs[i].msg_off = x.msg_off;
      sigs[i].msg_sz = x.msg_sz;
      sigs[i].sig_off = x.sig_off + 64u * j;
      sigs[i].pub_off = x.pub_off + 32u * j;
      if (perm) perm[i] = s0 + j;
    }
  }
  return (int64_t)ns;
}

/* RAII device buffer (diagnostics) */
struct DevBuf {
  void *p = nullptr;
  ~DevBuf() { if (p) (void)hipFree(p); }
};

/* (Re)size the per-lane workspace to cover n_sig signatures. */
int ensure_ws(fdgpu_engine *e, uint64_t n_sig) {
  if (n_sig <= e->ws_sig && e->d_ws) return FDGPU_OK;
  if (e->d_ws) { (void)hipFree(e->d_ws); e->d_ws = nullptr; }
  e->ws_bytes = fdgpu_ws_bytes(n_sig ? n_sig : 1);
  if (hipMalloc((void **)&e->d_ws, e->ws_bytes) != hipSuccess) {
    set_err("workspace alloc (%zu bytes)", e->ws_bytes); e->ws_sig = 0; return FDGPU_ERR_DEVICE;
  }
  e->ws_sig = n_sig ? n_sig : 1;
  return FDGPU_OK;
}

}  // namespace

/* Host regions registered for direct DMA (hipHostRegister, portable to every
   device), reference-counted across the engines that registered them. */
namespace {
std::mutex g_reg_mu;

/* The fixed-base comb table is a device constant (67 MB): one copy per
   device, shared by every engine opened on it (refcounted), so engines of
   several verify tiles on one GPU read the same lines from the Infinity
   Cache instead of each streaming its own copy. */
std::mutex g_btab_mu;
std::map<int, std::pair<uint32_t *, int>> g_btab;

uint32_t *btab_acquire(int device, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_btab_mu);
  auto it = g_btab.find(device);
  if (it != g_btab.end()) { it->second.second++; return it->second.first; }
  uint32_t *p = nullptr;
  if (hipMalloc((void **)&p, fdgpu_btab_bytes()) != hipSuccess) { set_err("btab alloc"); return nullptr; }
  if (fdgpu_btab_build(p, st) != hipSuccess) { (void)hipFree(p); set_err("fixed-base table build failed"); return nullptr; }
  g_btab[device] = {p, 1};
  return p;
}

void btab_release(int device, uint32_t *p) {
  std::lock_guard<std::mutex> lk(g_btab_mu);
  auto it = g_btab.find(device);
  if (it == g_btab.end() || it->second.first != p) return;
  if (--it->second.second == 0) { (void)hipFree(p); g_btab.erase(it); }
}
/* pinned host regions: page-aligned base -> end, references over every
   engine's registrations, and the device-side address of base (regions are
   mapped, so kernels read them in place: fdgpu_submit_frags_io) */
struct GReg { uintptr_t end; int refs; uintptr_t dbase; };
std::map<uintptr_t, GReg> g_regions;

/* the engine's registration covering [p, p + sz), or null */
const fdgpu_engine::Reg *region_of(const fdgpu_engine *e, uintptr_t p, uint64_t sz) {
  for (const auto &r : e->regions)
    if (p >= r.base && p + sz <= r.end) return &r;
  return nullptr;
}

bool region_covers(const fdgpu_engine *e, const uint8_t *p, uint64_t sz) {
  const uintptr_t a = (uintptr_t)p;
  for (const auto &r : e->regions)
    if (a >= r.base && a + sz <= r.end) return true;
  return false;
}

/* drop one reference to the pinned region at base */
void region_release(int device, uintptr_t base) {
  std::lock_guard<std::mutex> rk(g_reg_mu);
  auto it = g_regions.find(base);
  if (it == g_regions.end()) return;
  if (--it->second.refs == 0) {
    (void)hipSetDevice(device);
    (void)hipHostUnregister((void *)base);
    g_regions.erase(it);
  }
}
}  // namespace

static bool bucket(const fdgpu_engine_t *e) { return !(e->cfg.flags & FDGPU_FLAG_NO_BUCKET); }
/* the kernels' flags for this engine's configuration */
static uint32_t kflags(const fdgpu_engine_t *e) {
  return ((e->cfg.flags & FDGPU_FLAG_REF_MAPPING) ? FDGPU_FLAG_REF_MAP : 0u) |
         ((e->cfg.flags & FDGPU_FLAG_SPREAD) ? FDGPU_FLAG_KSPREAD : 0u) |
         ((e->cfg.flags & FDGPU_FLAG_FULL_PATH) ? FDGPU_FLAG_KFULL : 0u) |
         ((e->cfg.flags & FDGPU_FLAG_KEY_CACHE) ? FDGPU_FLAG_KCACHE : 0u) |
         ((e->cfg.flags & FDGPU_FLAG_PAIR) && !(e->cfg.flags & FDGPU_FLAG_KEY_CACHE) ? FDGPU_FLAG_KPAIR : 0u);
}

/* FDGPU_FLAG_PAIR_AUTO: a ring batch takes the two-lane kernel while the
   signatures of the engine's running batches and its own (launch bounds:
   a gathered batch's count is known only on the device), two lanes each,
   leave part of the chip's resident lanes idle (256 CUs x 4 SIMDs x 2 waves
   x 64 = 131,072): a wave's lifetime is then the batch's latency
   (profiles/r04/pair_rocprof.txt: 0.73x the one-lane kernel's time at 4-16 K
   signatures, 0.76x at 32 K; pair_probe.jsonl: 1.2x at 64 K, where two lanes
   per signature fill the chip).  A loaded engine keeps the one-lane kernel,
   which does ~1.4x less work per signature. */
static constexpr uint64_t FDGPU_PAIR_AUTO_SIGS = 49152;

/* FDGPU_FLAG_SPREAD_AUTO: a ring batch's verify blocks take one CU each
   (FDGPU_FLAG_KSPREAD: dynamic LDS that leaves no room for a second block)
   while its lanes and those of the engine's running batches fit the chip
   one block per CU (256 CUs x 256 lanes).  Concurrent launches from other
   streams otherwise stack two blocks on a CU while other CUs idle: four
   16 K launches at once verify 82 M sigs/s spread against 55 M packed, but
   spread caps the chip at ~89 M where packing reaches 106 M with 12+
   launches (profiles/r04/spread.md). */
static constexpr uint64_t FDGPU_SPREAD_AUTO_LANES = 65536;

/* The auto flags can weigh the running batches of every engine open on the
   device, not only the caller's: each verify tile has an engine of its own,
   and two tiles at capacity each saw about half the chip's load -- each
   kept spreading its verifies one block per CU (and taking the two-lane
   kernel) while the chip was full.  Measured, that view is the worse one:
   two tiles at capacity 58.8 vs 60.1 M txn/s and, paced at 24 M, p50 / p99
   batch latency 1.31 / 1.78 vs 0.97 / 1.07 ms (profiles/r05/auto_scope.md),
   so the per-engine view stays the default and FDGPU_AUTO_SCOPE=device
   selects this one.  Other engines' slots are read without their locks:
   the fields are atomics, and a stale view only shifts the estimate by a
   batch. */
namespace {
std::mutex g_dev_mu;
std::map<int, std::vector<fdgpu_engine_t *>> g_dev_eng;
const bool g_auto_engine_scope = !(getenv("FDGPU_AUTO_SCOPE") && !strcmp(getenv("FDGPU_AUTO_SCOPE"), "device"));

/* signatures and lanes of o's running batches (s excluded) into load, lanes */
void running_load(const fdgpu_engine_t *o, const Slot *s, uint64_t &load, uint64_t &lanes) {
  for (const auto &c : o->slots) {
    if (&c == s || __atomic_load_n(&c.ticket, __ATOMIC_RELAXED) < 0) continue;
    if (o->flag_poll && __atomic_load_n(c.h_flag, __ATOMIC_ACQUIRE) == __atomic_load_n(&c.flag_seq, __ATOMIC_RELAXED))
      continue;                                                      /* complete, not yet polled */
    load += __atomic_load_n(&c.k_sigs, __ATOMIC_RELAXED);
    lanes += __atomic_load_n(&c.k_lanes, __ATOMIC_RELAXED);
  }
}
}  // namespace

/* the kernel flags of slot s's ring batch of n_sig signatures (ring_mu held) */
static uint32_t ring_kflags(fdgpu_engine_t *e, Slot *s, uint64_t n_sig) {
  uint32_t f = kflags(e);
  const uint64_t auto_flags = e->cfg.flags & (FDGPU_FLAG_PAIR_AUTO | FDGPU_FLAG_SPREAD_AUTO);
  st_rlx(s->k_sigs, n_sig);
  if (auto_flags && !(f & FDGPU_FLAG_KCACHE)) {
    uint64_t load = n_sig, lanes = 0;
    if (g_auto_engine_scope) {
      running_load(e, s, load, lanes);
    } else {
      std::lock_guard<std::mutex> dk(g_dev_mu);
      for (const fdgpu_engine_t *o : g_dev_eng[e->device]) running_load(o, s, load, lanes);
    }
    if ((auto_flags & FDGPU_FLAG_PAIR_AUTO) && load <= FDGPU_PAIR_AUTO_SIGS) f |= FDGPU_FLAG_KPAIR;
    lanes += (f & FDGPU_FLAG_KPAIR) ? 2 * n_sig : n_sig;
    if ((auto_flags & FDGPU_FLAG_SPREAD_AUTO) && lanes <= FDGPU_SPREAD_AUTO_LANES) f |= FDGPU_FLAG_KSPREAD;
  }
  st_rlx(s->k_lanes, (f & FDGPU_FLAG_KPAIR) ? 2 * n_sig : n_sig);
  return f;
}

extern "C" {

char const *fdgpu_last_error(void) { return g_err.c_str(); }

int fdgpu_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n < 1) { (void)hipGetLastError(); return -1; }
  return n;
}

fdgpu_engine_t *fdgpu_engine_open(int device, fdgpu_cfg_t const *cfg_in) {
  fdgpu_cfg_t cfg{};
  if (cfg_in) cfg = *cfg_in;
  if (!cfg.max_txn) cfg.max_txn = 1u << 16;
  /* a parsed transaction carries at most 12 signatures (FD_TXN_ACTUAL_SIG_MAX,
     fd_txn.h:68); batches whose signatures exceed max_sig are rejected */
  if (!cfg.max_sig) cfg.max_sig = cfg.max_txn * 12;
  if (!cfg.max_arena) cfg.max_arena = cfg.max_txn * 1232ull;
  if (!cfg.ring_depth) cfg.ring_depth = 2;
  if (cfg.max_arena > 0xFFFFFFF0ull || cfg.max_sig > 0xFFFFFFF0ull || cfg.max_txn > 0xFFFFFFF0ull) {
    set_err("batch limits exceed 32-bit offsets");
    return nullptr;
  }
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev), nullptr);
  if (device < 0 || device >= ndev) { set_err("device %d not present (%d devices)", device, ndev); return nullptr; }
  HIPCHK(hipSetDevice(device), nullptr);
  fdgpu_engine *e = new fdgpu_engine();
  e->device = device;
  e->cfg = cfg;
  auto fail = [&]() -> fdgpu_engine_t * { fdgpu_engine_close(e); return nullptr; };
  if (hipStreamCreateWithFlags(&e->compute, hipStreamNonBlocking) != hipSuccess) { set_err("stream"); return fail(); }
  if (!(e->d_btab = btab_acquire(device, e->compute))) return fail();
  int bpcu = 0;
  hipDeviceProp_t prop;
  if (fdgpu_verify_occupancy(&bpcu) != hipSuccess || bpcu < 1) bpcu = 1;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) { set_err("props"); return fail(); }
  e->resident_blocks = (uint32_t)(bpcu * prop.multiProcessorCount);
  {
    std::random_device rd;                     /* per-engine key-cache seed: crafted keys cannot target it */
    e->kc_seed = (((uint64_t)rd() << 32) | rd()) | 1u;
  }
  e->slots.resize(cfg.ring_depth);
  for (auto &s : e->slots) if (!slot_alloc(s, cfg)) return fail();
  if (hipStreamSynchronize(e->compute) != hipSuccess) { set_err("btab init failed"); return fail(); }
  /* completion words: probe that a stream write reaches pinned host memory
     (FDGPU_POLL_EVENT=1 keeps hipEventQuery polling) */
  {
    const char *pe = getenv("FDGPU_POLL_EVENT"), *df = getenv("FDGPU_DEBUG_DROP_FLAG");
    e->drop_flag = df && df[0] == '1';
    const char *fm = getenv("FDGPU_DEBUG_FAIL_MERGE");
    e->fail_merge_at = fm ? (uint32_t)atoi(fm) : 0u;
    Slot &s0 = e->slots[0];
    if (!(pe && pe[0] == '1') && hipStreamWriteValue32(s0.stream, s0.d_flag, 0x5a5a5a5au, 0) == hipSuccess &&
        hipStreamSynchronize(s0.stream) == hipSuccess)
      e->flag_poll = __atomic_load_n(s0.h_flag, __ATOMIC_ACQUIRE) == 0x5a5a5a5au;
    (void)hipGetLastError();
    *s0.h_flag = 0;
  }
  if (cfg.flags & FDGPU_FLAG_MERGE) {
    /* two merge streams (a merged verify's tail overlaps the next one's
       start); a table is reused only after 2 x ring_depth + 2 launches on its
       stream, by when the launch that read it has finished (every launch in
       flight holds a batch not yet complete, so at most ring_depth are) */
    const char *ms = getenv("FDGPU_MERGE_STREAMS");
    const uint32_t nms = ms && ms[0] == '1' ? 1u : 2u;
    e->merge_tabs = 2 * cfg.ring_depth + 2;
    e->merges.resize(nms);
    for (auto &m : e->merges) {
      if (hipStreamCreateWithFlags(&m.stream, hipStreamNonBlocking) != hipSuccess ||
          hipHostMalloc((void **)&m.h_flag, 64, hipHostMallocDefault) != hipSuccess ||
          hipHostGetDevicePointer((void **)&m.d_flag, m.h_flag, 0) != hipSuccess ||
          hipHostMalloc((void **)&m.h_tab, (size_t)e->merge_tabs * cfg.ring_depth * sizeof(fdgpu_mbatch_t),
                        hipHostMallocDefault) != hipSuccess ||
          hipHostGetDevicePointer((void **)&m.d_tab, m.h_tab, 0) != hipSuccess) {
        set_err("merge stream");
        return fail();
      }
      *m.h_flag = 0;
      m.ev.resize(e->merge_tabs);
      for (auto &ev : m.ev)
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) { set_err("merge event"); return fail(); }
    }
    e->pending.reserve(cfg.ring_depth);
  }
  {
    std::lock_guard<std::mutex> dk(g_dev_mu);
    g_dev_eng[device].push_back(e);
  }
  return e;
}

void fdgpu_engine_close(fdgpu_engine_t *e) {
  if (!e) return;
  {
    std::lock_guard<std::mutex> dk(g_dev_mu);                /* no other engine reads its slots from here on */
    auto &v = g_dev_eng[e->device];
    v.erase(std::remove(v.begin(), v.end(), e), v.end());
  }
  if (g_sp_on && g_sp_calls)
    fprintf(stderr, "[fdgpu submit_frags_io] calls %llu frags %llu: loop %.1f us/call, enqueue %.1f us/call\n",
            (unsigned long long)g_sp_calls.load(), (unsigned long long)g_sp_frags.load(),
            g_sp_loop.load() / 1e3 / g_sp_calls.load(), g_sp_enq.load() / 1e3 / g_sp_calls.load());
  (void)hipSetDevice(e->device);
  if (e->compute) (void)hipStreamSynchronize(e->compute);
  for (auto &m : e->merges) if (m.stream) (void)hipStreamSynchronize(m.stream);
  for (auto &s : e->slots) { if (s.stream) (void)hipStreamSynchronize(s.stream); slot_free(s); }
  for (auto b : e->big) if (b) { (void)hipStreamSynchronize(b); (void)hipStreamDestroy(b); }
  for (auto &m : e->merges) {
    for (auto ev : m.ev) if (ev) (void)hipEventDestroy(ev);
    if (m.h_tab) (void)hipHostFree(m.h_tab);
    if (m.h_flag) (void)hipHostFree(m.h_flag);
    if (m.stream) (void)hipStreamDestroy(m.stream);
  }
  for (auto &r : e->regions) region_release(e->device, r.base);
  for (auto st : e->batch_streams) (void)hipStreamSynchronize(st);   /* btab is read there */
  if (e->d_btab) btab_release(e->device, e->d_btab);
  if (e->d_ws) (void)hipFree(e->d_ws);
  if (e->d_scratch_codes) (void)hipFree(e->d_scratch_codes);
  if (e->compute) (void)hipStreamDestroy(e->compute);
  delete e;
}

int fdgpu_engine_reserve(fdgpu_engine_t *e, uint64_t n_sig) {
  if (!e) return FDGPU_ERR_INVAL;
  if (!n_sig) n_sig = e->cfg.max_sig;
  if (n_sig > e->cfg.max_sig) { set_err("reserve beyond max_sig"); return FDGPU_ERR_INVAL; }
  std::lock_guard<std::mutex> lk(e->ring_mu);
  for (auto &s : e->slots) if (s.ticket >= 0 || s.staged) { set_err("a slot holds a batch"); return FDGPU_ERR_FULL; }
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  const uint64_t n = e->cfg.max_txn, res = ((n + 63) & ~63ull) + n * 10;    /* a gathered batch's results */
  for (auto &s : e->slots)
    if (!slot_ws(s, n_sig) || !slot_frag_bufs(s, e->cfg, res) || !slot_io_bufs(s, e->cfg)) return FDGPU_ERR_DEVICE;
  return FDGPU_OK;
}

int fdgpu_engine_info(fdgpu_engine_t *e, uint32_t *grid_blocks, uint32_t *block_threads, uint64_t *ws_bytes) {
  if (!e) return FDGPU_ERR_INVAL;
  if (grid_blocks) *grid_blocks = e->resident_blocks;
  if (block_threads) *block_threads = FDGPU_BLOCK;
  if (ws_bytes) *ws_bytes = e->ws_bytes;
  return FDGPU_OK;
}

/* ws: a workspace for n_sig signatures, or NULL for the engine's compute
   workspace (grown on demand; callers on other streams synchronise first). */
static int enqueue_verify(fdgpu_engine_t *e, const uint8_t *d_arena, const fdgpu_sig_desc_t *d_sigs,
                          const uint32_t *d_perm, uint64_t n_sig, const fdgpu_txn_desc_t *d_txns, uint64_t n_txn,
                          int8_t *d_sig_codes, int8_t *d_txn_codes, hipStream_t st, uint32_t *ws = nullptr,
                          uint32_t flags = ~0u) {
  if (flags == ~0u) flags = kflags(e);
  if (!ws && n_sig > e->ws_sig) {
    HIPCHK(hipStreamSynchronize(st), FDGPU_ERR_DEVICE);
    HIPCHK(hipStreamSynchronize(e->compute), FDGPU_ERR_DEVICE);
    int rc = ensure_ws(e, n_sig);
    if (rc) return rc;
  }
  HIPCHK(fdgpu_launch_verify_sigs(d_arena, d_sigs, (uint32_t)n_sig, d_perm, e->d_btab, ws ? ws : e->d_ws, d_sig_codes,
                                  flags, st, nullptr, e->resident_blocks, e->kc_seed),
         FDGPU_ERR_DEVICE);
  HIPCHK(fdgpu_launch_combine(d_txns, (uint32_t)n_txn, d_sig_codes, d_txn_codes, nullptr, st), FDGPU_ERR_DEVICE);
  return FDGPU_OK;
}

/* A ring batch of at least this many signatures fills every resident lane
   of the chip (256 CUs x 4 SIMDs x 2 waves x 64 = 131,072) on its own.  Its
   verify runs on one of the engine's two big-batch streams, in turn, after
   its uploads (an event wait), and its read-back waits for it: at most two
   such verifies overlap (the next one's waves fill the tail the previous
   one leaves, as the device-resident line's two queues do), and the next
   slots' uploads run under them.  On their own slot streams three 1 M
   batches ran in lockstep -- three uploads at once with the GPU idle, then
   three verifies at once -- 11.6-12.0 ms a batch from a registered arena
   against 10.3 staged (rocprofv3 with --memory-copy-trace,
   profiles/r05/host_fed_lockstep.md). */
static constexpr uint64_t FDGPU_BIG_SIGS = 262144;

namespace {
int64_t expand_par(uint64_t arena_sz, const fdgpu_txn_t *txns, uint64_t txn_cnt, uint64_t max_sig,
                   fdgpu_sig_desc_t *sigs, fdgpu_txn_desc_t *tds, uint32_t *perm);
}

/* Enqueue the batch already in slot s's pinned arena (arena_sz bytes). */
/* `uploaded` = bytes of the arena whose host->device copy is already queued on
   the slot's stream (fdgpu_submit overlaps its staging memcpy with the copy) */
/* src != NULL: the arena lies in a registered host region and is uploaded
   straight from there (no staging copy); its bytes must stay unchanged until
   the batch is polled. */
static int64_t submit_slot(fdgpu_engine_t *e, Slot *s, uint64_t arena_sz, fdgpu_txn_t const *txns, uint64_t txn_cnt,
                           uint64_t uploaded = 0, const uint8_t *src = nullptr, uint64_t t_stage = 0) {
  uint32_t *perm = bucket(e) ? s->h_perm : nullptr;
  /* a registered arena's DMA is queued first, so it runs under the
     descriptor expansion (an arena expand() rejects leaves the slot free; the
     next batch's copies, later on the same stream, overwrite it) */
  if (src && arena_sz) HIPCHK(hipMemcpyAsync(s->d_arena, src, arena_sz, hipMemcpyHostToDevice, s->stream), FDGPU_ERR_DEVICE);
  const uint64_t t0 = sp_now();
  const int64_t ns = expand_par(arena_sz, txns, txn_cnt, e->cfg.max_sig, s->h_sigs, s->h_txns, perm);
  if (ns < 0) return FDGPU_ERR_INVAL;
  const uint64_t t1 = sp_now();
  struct Rec {                                  /* the call's times into the ring, on every return */
    uint64_t st, t0, t1;
    ~Rec() {
      const uint64_t k = g_st_n.fetch_add(1, std::memory_order_relaxed) % FDGPU_ST_RING;
      g_st[k][0].store(st, std::memory_order_relaxed);
      g_st[k][1].store(t1 - t0, std::memory_order_relaxed);
      g_st[k][2].store(sp_now() - t1, std::memory_order_relaxed);
    }
  } rec{t_stage, t0, t1};
  if (!slot_ws(*s, (uint64_t)ns)) return FDGPU_ERR_DEVICE;
  if (src) {
    /* the slack past a registered arena is left as it is: the SHA block
       loads mask every byte past the message (msg_block), so only its
       presence matters.  Zeroing it on the device cost a kernel (a fill, or
       the blit of a small copy) queued behind the upload, which waits for a
       CU slot the running verify holds -- the batch's descriptor copies and
       verify waited behind it, ~7 ms a 1 M batch
       (profiles/r05/host_fed/registered_slack.md) */
  } else {
    memset(s->h_arena + arena_sz, 0, FDGPU_ARENA_SLACK);
    const size_t asz = arena_sz + FDGPU_ARENA_SLACK - uploaded;
    HIPCHK(hipMemcpyAsync(s->d_arena + uploaded, s->h_arena + uploaded, asz, hipMemcpyHostToDevice, s->stream),
           FDGPU_ERR_DEVICE);
  }
  if (ns) HIPCHK(hipMemcpyAsync(s->d_sigs, s->h_sigs, (size_t)ns * sizeof(fdgpu_sig_desc_t), hipMemcpyHostToDevice, s->stream), FDGPU_ERR_DEVICE);
  if (ns && perm) HIPCHK(hipMemcpyAsync(s->d_perm, perm, (size_t)ns * sizeof(uint32_t), hipMemcpyHostToDevice, s->stream), FDGPU_ERR_DEVICE);
  if (txn_cnt) HIPCHK(hipMemcpyAsync(s->d_txns, s->h_txns, txn_cnt * sizeof(fdgpu_txn_desc_t), hipMemcpyHostToDevice, s->stream), FDGPU_ERR_DEVICE);
  /* copies, kernels and the code read-back of a slot run in order on the
     slot's own stream with the slot's own workspace, so the ring's batches
     overlap each other on the GPU (a 64K-signature batch fills only half of
     the resident wave slots) */
  hipStream_t vs = s->stream;
  if ((uint64_t)ns >= FDGPU_BIG_SIGS && !g_big_off) {
    for (auto &b : e->big)
      if (!b) HIPCHK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking), FDGPU_ERR_DEVICE);
    vs = e->big[e->big_rr++ & 1u];
    HIPCHK(hipEventRecord(s->h2d_done, s->stream), FDGPU_ERR_DEVICE);
    HIPCHK(hipStreamWaitEvent(vs, s->h2d_done, 0), FDGPU_ERR_DEVICE);
  }
  int rc = enqueue_verify(e, s->d_arena, s->d_sigs, perm ? s->d_perm : nullptr, (uint64_t)ns, s->d_txns, txn_cnt,
                          s->d_sig_codes, s->d_txn_codes, vs, s->d_ws, ring_kflags(e, s, (uint64_t)ns));
  if (rc) return rc;
  if (vs != s->stream) {
    HIPCHK(hipEventRecord(s->comp_done, vs), FDGPU_ERR_DEVICE);
    HIPCHK(hipStreamWaitEvent(s->stream, s->comp_done, 0), FDGPU_ERR_DEVICE);
  }
  if (txn_cnt) HIPCHK(hipMemcpyAsync(s->h_codes, s->d_txn_codes, txn_cnt, hipMemcpyDeviceToHost, s->stream), FDGPU_ERR_DEVICE);
  slot_flag_next(s);
  if (e->flag_poll && !e->drop_flag) HIPCHK(hipStreamWriteValue32(s->stream, s->d_flag, s->flag_seq, 0), FDGPU_ERR_DEVICE);
  HIPCHK(hipEventRecord(s->done, s->stream), FDGPU_ERR_DEVICE);
  s->staged = false;
  st_rlx(s->held, false);
  st_rlx(s->polls, 0u);
  s->frag = false;
  s->io = false;
  st_rlx(s->ticket, e->next_ticket++);
  s->txn_cnt = txn_cnt;
  return s->ticket;
}

static Slot *free_slot(fdgpu_engine_t *e) {
  for (auto &c : e->slots) if (c.ticket < 0 && !c.staged) return &c;
  return nullptr;
}

/* Copy a caller's arena into the slot's pinned buffer.  Large arenas are
   split over FDGPU_COPY_THREADS host threads; each queues its part's upload on
   the slot stream as soon as its memcpy is done, so the PCIe copy runs under
   the rest of the staging (one core's memcpy bandwidth, ~15 GB/s, otherwise
   bounds submit()).  Returns the bytes already queued for upload, or
   UINT64_MAX on a HIP error.  An arena that expand() later rejects leaves the
   slot free; its stale upload is overwritten by the next batch's copies,
   which are ordered after it on the same stream. */
#ifndef FDGPU_COPY_THREADS_N
#define FDGPU_COPY_THREADS_N 4                 /* A/B builds may change it */
#endif
static constexpr unsigned FDGPU_COPY_THREADS = FDGPU_COPY_THREADS_N;
static constexpr uint64_t FDGPU_COPY_SPLIT_MIN = 4ull << 20;
/* FDGPU_COPY_CHUNK_MB overrides the upload piece (A/B; 0: one piece per thread) */
const uint64_t FDGPU_COPY_CHUNK = [] {
  const char *v = getenv("FDGPU_COPY_CHUNK_MB");
  const long long m = v ? atoll(v) : 16;
  return m > 0 ? (uint64_t)m << 20 : UINT64_MAX;
}();

char const *fdgpu_build_info(void) {
  static thread_local char buf[512];
  char kb[256];
  const int kprod = fdgpu_kernel_build_info(kb, sizeof kb);
  const char *df = getenv("FDGPU_DEBUG_DROP_FLAG");      /* fault injection: completion flags dropped */
  const char *fm = getenv("FDGPU_DEBUG_FAIL_MERGE");     /* fault injection: a merge launch fails */
  const int drop = df && df[0] == '1', fail_merge = fm ? atoi(fm) : 0;
  const int prod = kprod && FDGPU_COPY_THREADS_N == 4 && !drop && !fail_merge;
  snprintf(buf, sizeof buf, "{%s,\"copy_threads\":%d,\"debug_drop_flag\":%d,\"debug_fail_merge\":%d,\"product\":%d}",
           kb, (int)FDGPU_COPY_THREADS_N, drop, fail_merge, prod);
  return buf;
}

}  // extern "C"

/* The staging helpers: FDGPU_COPY_THREADS - 1 process-wide threads started
   on first use and kept (a thread created per submit costs tens of
   microseconds and was a visible share of a batch's latency tail). */
namespace {
struct CopyPool {
  std::mutex mu;
  std::condition_variable cv, done_cv;
  std::vector<std::function<void()>> jobs;
  uint64_t pending = 0;
  std::vector<std::thread> th;
  CopyPool() {
    for (unsigned i = 1; i < FDGPU_COPY_THREADS; i++)
      th.emplace_back([this]() {
        for (;;) {
          std::function<void()> job;
          {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [this]() { return !jobs.empty(); });
            job = std::move(jobs.back());
            jobs.pop_back();
          }
          job();
          std::lock_guard<std::mutex> lk(mu);
          if (--pending == 0) done_cv.notify_all();
        }
      });
    for (auto &t : th) t.detach();           /* live for the process */
  }
  /* runs fns[1..] on the pool and fns[0] here; returns when all are done */
  void run(std::vector<std::function<void()>> &fns) {
    {
      std::lock_guard<std::mutex> lk(mu);
      for (size_t i = 1; i < fns.size(); i++) { jobs.push_back(fns[i]); pending++; }
    }
    cv.notify_all();
    fns[0]();
    std::unique_lock<std::mutex> lk(mu);
    done_cv.wait(lk, [this]() { return pending == 0; });
  }
};
CopyPool &copy_pool() {
  static CopyPool *p = new CopyPool;         /* never destroyed: its threads outlive main */
  return *p;
}
std::mutex g_stage_mu;                       /* one staging at a time uses the pool */

/* expand() over FDGPU_COPY_THREADS parts of the transactions at once, for
   the large batches whose single-threaded expansion (~3 ns a txn, 3 ms for
   1 M) sat on the submitting thread beside the staging copy: pass 1 counts
   and validates each part (signatures, block-count groups, the first bad
   txn), pass 2 writes each part's descriptors at its prefix offsets, so the
   output -- sig0s, descriptors, the stable block-count grouping and its
   permutation -- is byte-identical to expand()'s, and so is the error
   (the first failing txn in order, of either kind). */
static constexpr uint64_t FDGPU_EXPAND_SPLIT_MIN = 65536;

int64_t expand_par(uint64_t arena_sz, const fdgpu_txn_t *txns, uint64_t txn_cnt, uint64_t max_sig,
                   fdgpu_sig_desc_t *sigs, fdgpu_txn_desc_t *tds, uint32_t *perm) {
  if (txn_cnt < FDGPU_EXPAND_SPLIT_MIN) return expand(arena_sz, txns, txn_cnt, max_sig, sigs, tds, perm);
  constexpr unsigned T = FDGPU_COPY_THREADS;
  struct Part {
    uint64_t lo = 0, hi = 0, ns = 0, bad = UINT64_MAX;
    uint64_t grp[FDGPU_NBLK_GROUPS] = {};
  } part[T];
  const uint64_t per = (txn_cnt + T - 1) / T;
  for (unsigned k = 0; k < T; k++) {
    part[k].lo = std::min<uint64_t>(txn_cnt, k * per);
    part[k].hi = std::min<uint64_t>(txn_cnt, part[k].lo + per);
  }
  std::vector<std::function<void()>> fns;
  for (unsigned k = 0; k < T; k++)
    fns.push_back([&, k]() {
      Part &q = part[k];
      for (uint64_t t = q.lo; t < q.hi; t++) {
        const fdgpu_txn_t &x = txns[t];
        const uint32_t cnt = x.sig_cnt;
        tds[t].sig0 = (uint32_t)q.ns;                        /* part-relative until pass 2 */
        tds[t].sig_cnt = cnt;
        if (cnt == 0 || cnt > 16) { tds[t].sig_cnt = 0; continue; }
        if ((uint64_t)x.msg_off + x.msg_sz > arena_sz || (uint64_t)x.sig_off + 64ull * cnt > arena_sz ||
            (uint64_t)x.pub_off + 32ull * cnt > arena_sz) { q.bad = t; return; }
        if (perm) q.grp[std::min(hram_blocks(x.msg_sz), FDGPU_NBLK_GROUPS) - 1] += cnt;
        q.ns += cnt;
      }
    });
  {
    std::lock_guard<std::mutex> lk(g_stage_mu);
    copy_pool().run(fns);
  }
  /* the first failure in transaction order: a part's bad descriptor, or the
     txn at which the running count passes max_sig (expand()'s two checks) */
  uint64_t base = 0;
  for (unsigned k = 0; k < T; k++) {
    const Part &q = part[k];
    const uint64_t end = q.bad == UINT64_MAX ? q.hi : q.bad;
    if (base + q.ns > max_sig || q.bad != UINT64_MAX) {
      uint64_t ns = base;
      for (uint64_t t = q.lo; t < end; t++) {
        const uint32_t c = tds[t].sig_cnt;
        if (ns + c > max_sig) { set_err("batch exceeds max_sig (%llu)", (unsigned long long)max_sig); return -1; }
        ns += c;
      }
      if (q.bad != UINT64_MAX) {
        set_err("txn %llu: descriptor out of arena bounds", (unsigned long long)q.bad);
        return -1;
      }
    }
    base += q.ns;
  }
  uint64_t next[T][FDGPU_NBLK_GROUPS], sig_base[T];
  {
    uint64_t o = 0, gbase[FDGPU_NBLK_GROUPS], acc = 0;
    for (uint32_t g = 0; g < FDGPU_NBLK_GROUPS; g++) {
      gbase[g] = o;
      for (unsigned k = 0; k < T; k++) o += part[k].grp[g];
    }
    for (unsigned k = 0; k < T; k++) {
      sig_base[k] = acc;
      acc += part[k].ns;
      for (uint32_t g = 0; g < FDGPU_NBLK_GROUPS; g++) {
        next[k][g] = gbase[g];
        gbase[g] += part[k].grp[g];
      }
    }
  }
  fns.clear();
  for (unsigned k = 0; k < T; k++)
    fns.push_back([&, k]() {
      const Part &q = part[k];
      uint64_t *nx = next[k];
      for (uint64_t t = q.lo; t < q.hi; t++) {
        const fdgpu_txn_t &x = txns[t];
        const uint32_t s0 = tds[t].sig0 + (uint32_t)sig_base[k];
        tds[t].sig0 = s0;
        const uint32_t cnt = tds[t].sig_cnt;
        if (!cnt) continue;
        uint64_t *slot = perm ? &nx[std::min(hram_blocks(x.msg_sz), FDGPU_NBLK_GROUPS) - 1] : nullptr;
        for (uint32_t j = 0; j < cnt; j++) {
          const uint64_t i = slot ? (*slot)++ : (uint64_t)s0 + j;
          sigs[i].msg_off = x.msg_off;
          sigs[i].msg_sz = x.msg_sz;
          sigs[i].sig_off = x.sig_off + 64u * j;
          sigs[i].pub_off = x.pub_off + 32u * j;
          if (perm) perm[i] = s0 + j;
        }
      }
    });
  {
    std::lock_guard<std::mutex> lk(g_stage_mu);
    copy_pool().run(fns);
  }
  return (int64_t)base;
}
}  // namespace

extern "C" {

static uint64_t stage_arena(fdgpu_engine_t *e, Slot *s, uint8_t const *arena, uint64_t sz) {
  if (sz < FDGPU_COPY_SPLIT_MIN) {
    memcpy(s->h_arena, arena, sz);
    return 0;
  }
  const uint64_t part = ((sz + FDGPU_COPY_THREADS - 1) / FDGPU_COPY_THREADS + 63) & ~63ull;
  int err[FDGPU_COPY_THREADS] = {};
  std::vector<std::function<void()>> fns;
  for (unsigned i = 0; i < FDGPU_COPY_THREADS; i++)
    fns.push_back([&, i]() {
      const uint64_t off = (uint64_t)i * part;
      if (off >= sz) return;
      const uint64_t n = sz - off < part ? sz - off : part;
      if (hipSetDevice(e->device) != hipSuccess) { err[i] = 1; return; }
      /* in FDGPU_COPY_CHUNK pieces, each queued for upload as soon as it is
         copied: the DMA starts ~1 ms into the staging instead of after it
         (a 1 M batch's 364 MB: its uploads then end ~3 ms sooner) */
      for (uint64_t c = 0; c < n; c += FDGPU_COPY_CHUNK) {
        const uint64_t m = n - c < FDGPU_COPY_CHUNK ? n - c : FDGPU_COPY_CHUNK;
        memcpy(s->h_arena + off + c, arena + off + c, m);
        if (hipMemcpyAsync(s->d_arena + off + c, s->h_arena + off + c, m, hipMemcpyHostToDevice, s->stream) !=
            hipSuccess) { err[i] = 1; return; }
      }
    });
  {
    std::lock_guard<std::mutex> lk(g_stage_mu);
    copy_pool().run(fns);
  }
  for (unsigned i = 0; i < FDGPU_COPY_THREADS; i++)
    if (err[i]) { set_err("staging upload failed"); return UINT64_MAX; }
  return sz;
}

int64_t fdgpu_submit(fdgpu_engine_t *e, uint8_t const *arena, uint64_t arena_sz, fdgpu_txn_t const *txns,
                     uint64_t txn_cnt) {
  if (!e || (!arena && arena_sz) || (!txns && txn_cnt)) { set_err("null argument"); return FDGPU_ERR_INVAL; }
  if (arena_sz > e->cfg.max_arena || txn_cnt > e->cfg.max_txn) { set_err("batch exceeds engine limits"); return FDGPU_ERR_INVAL; }
  std::lock_guard<std::mutex> lk(e->ring_mu);
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  Slot *s = free_slot(e);
  if (!s) { set_err("all ring slots hold unpolled batches"); return FDGPU_ERR_FULL; }
  if (region_covers(e, arena, arena_sz)) return submit_slot(e, s, arena_sz, txns, txn_cnt, 0, arena);
  /* the slot's previous batch was polled, so its copies are complete */
  const uint64_t ts = sp_now();
  const uint64_t up = stage_arena(e, s, arena, arena_sz);
  if (up == UINT64_MAX) return FDGPU_ERR_DEVICE;
  return submit_slot(e, s, arena_sz, txns, txn_cnt, up, nullptr, sp_now() - ts);
}

uint64_t fdgpu_debug_submit_times(uint64_t *out, uint64_t max) {
  const uint64_t n = std::min<uint64_t>(g_st_n.load(), FDGPU_ST_RING), m = std::min(n, max);
  const uint64_t end = g_st_n.load();
  for (uint64_t i = 0; i < m; i++) {
    const uint64_t k = (end - m + i) % FDGPU_ST_RING;
    for (int j = 0; j < 3; j++) out[3 * i + j] = g_st[k][j].load(std::memory_order_relaxed);
  }
  return m;
}

double fdgpu_debug_h2d_gbps(fdgpu_engine_t *e, void const *src, uint64_t sz, int iters) {
  if (!e || !src || !sz || iters < 1 || sz > e->cfg.max_arena) { set_err("bad argument"); return -1.0; }
  std::lock_guard<std::mutex> lk(e->ring_mu);
  Slot *s = free_slot(e);
  if (!s) { set_err("all ring slots hold unpolled batches"); return -1.0; }
  HIPCHK(hipSetDevice(e->device), -1.0);
  hipEvent_t a, b;
  HIPCHK(hipEventCreate(&a), -1.0);
  if (hipEventCreate(&b) != hipSuccess) { (void)hipEventDestroy(a); set_err("event"); return -1.0; }
  double gbps = -1.0;
  float ms = 0.f;
  if (hipMemcpyAsync(s->d_arena, src, sz, hipMemcpyHostToDevice, s->stream) == hipSuccess &&   /* warm */
      hipEventRecord(a, s->stream) == hipSuccess) {
    bool ok = true;
    for (int i = 0; i < iters && ok; i++)
      ok = hipMemcpyAsync(s->d_arena, src, sz, hipMemcpyHostToDevice, s->stream) == hipSuccess;
    if (ok && hipEventRecord(b, s->stream) == hipSuccess && hipEventSynchronize(b) == hipSuccess &&
        hipEventElapsedTime(&ms, a, b) == hipSuccess && ms > 0.f)
      gbps = (double)sz * iters / (ms * 1e-3) / 1e9;
  }
  (void)hipGetLastError();
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  if (gbps < 0) set_err("h2d timing failed");
  return gbps;
}

uint8_t *fdgpu_stage_acquire(fdgpu_engine_t *e, uint64_t *cap) {
  if (!e) return nullptr;
  std::lock_guard<std::mutex> lk(e->ring_mu);
  for (auto &c : e->slots) if (c.staged) { set_err("a slot is already staged"); return nullptr; }
  Slot *s = free_slot(e);
  if (!s) { set_err("all ring slots hold unpolled batches"); return nullptr; }
  s->staged = true;
  if (cap) *cap = e->cfg.max_arena;
  return s->h_arena;
}

int64_t fdgpu_stage_submit(fdgpu_engine_t *e, uint64_t arena_sz, fdgpu_txn_t const *txns, uint64_t txn_cnt) {
  if (!e || (!txns && txn_cnt)) { set_err("null argument"); return FDGPU_ERR_INVAL; }
  std::lock_guard<std::mutex> lk(e->ring_mu);
  Slot *s = nullptr;
  for (auto &c : e->slots) if (c.staged) { s = &c; break; }
  if (!s) { set_err("no staged slot"); return FDGPU_ERR_INVAL; }
  if (arena_sz > e->cfg.max_arena || txn_cnt > e->cfg.max_txn) { set_err("batch exceeds engine limits"); return FDGPU_ERR_INVAL; }
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  return submit_slot(e, s, arena_sz, txns, txn_cnt);
}

namespace {
int merge_kick(fdgpu_engine_t *e, bool force);
}

static int poll_slot(fdgpu_engine_t *e, int64_t ticket, int8_t *txn_codes, int blocking, bool keep,
                     uint8_t *trailers = nullptr, uint64_t *tags = nullptr, uint16_t *out_szs = nullptr) {
  if (!e) return FDGPU_ERR_INVAL;
  /* a batch still on the device is answered without the ring lock: the
     caller owns its ticket's slot until a poll returns it done, so the slot's
     ticket and completion word are stable here; the runtime check below
     (every 256th poll) and everything else take the lock */
  bool counted = false;                        /* this poll already counted in the slot's polls */
  if (!blocking && e->flag_poll && e->merges.empty() && ticket >= 0)
    for (auto &c : e->slots)
      if (__atomic_load_n(&c.ticket, __ATOMIC_RELAXED) == ticket) {
        if (!__atomic_load_n(&c.held, __ATOMIC_RELAXED) &&
            __atomic_load_n(c.h_flag, __ATOMIC_ACQUIRE) != __atomic_load_n(&c.flag_seq, __ATOMIC_RELAXED)) {
          counted = true;
          if ((__atomic_add_fetch(&c.polls, 1u, __ATOMIC_RELAXED) & 255u) != 0) return FDGPU_PENDING;
        }
        break;
      }
  std::unique_lock<std::mutex> lk(e->ring_mu);
  Slot *s = nullptr;
  for (auto &c : e->slots) if (c.ticket == ticket && ticket >= 0 && !c.held) { s = &c; break; }
  if (!s) { set_err("unknown ticket %lld", (long long)ticket); return FDGPU_ERR_TICKET; }
  if (s->failed) {                             /* its merged verify was never queued (merge_kick) */
    s->failed = false;
    st_rlx(s->ticket, (int64_t)-1);
    set_err("ticket %lld: its verify could not be queued", (long long)ticket);
    return FDGPU_ERR_DEVICE;
  }
  if (!e->pending.empty()) {                   /* FDGPU_FLAG_MERGE: verifies waiting for a merge stream */
    HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
    const int rc = merge_kick(e, blocking && s->vpending);
    if (rc) return rc;
    if (s->vpending) return FDGPU_PENDING;     /* non-blocking: not even launched */
  }
  if (blocking) {
    HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
    lk.unlock();                               /* the slot is this caller's until it is polled */
    HIPCHK(hipEventSynchronize(s->done), FDGPU_ERR_DEVICE);
    lk.lock();
  } else if (e->flag_poll) {
    /* the stream wrote flag_seq after the codes' read-back completed.  A
       stream that failed never writes it, so an unanswered poll asks the
       runtime now and then -- every 256th poll once 1 ms has passed since the
       last question (runtime queries from several tile threads contend):
       an error ends the wait (the tile stops instead of polling forever), a
       completed event means the batch is done. */
    if (__atomic_load_n(s->h_flag, __ATOMIC_ACQUIRE) != s->flag_seq) {
      if (!counted && (__atomic_add_fetch(&s->polls, 1u, __ATOMIC_RELAXED) & 255u) != 0) return FDGPU_PENDING;
      const uint64_t now = sp_now();
      if (now - s->last_query < 1000000ull) return FDGPU_PENDING;
      s->last_query = now;
      HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
      const hipError_t q = hipEventQuery(s->done);
      if (q == hipErrorNotReady) return FDGPU_PENDING;
      HIPCHK(q, FDGPU_ERR_DEVICE);
    }
  } else {
    HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
    hipError_t q = hipEventQuery(s->done);
    if (q == hipErrorNotReady) return FDGPU_PENDING;
    HIPCHK(q, FDGPU_ERR_DEVICE);
  }
  if (s->io) {                                 /* [codes][tags][out sizes] */
    const uint64_t n = s->txn_cnt, cb = (n + 63) & ~63ull;
    if (txn_codes && n) memcpy(txn_codes, s->h_tr, n);
    if (tags && n) memcpy(tags, s->h_tr + cb, n * 8);
    if (out_szs && n) memcpy(out_szs, s->h_tr + cb + n * 8, n * 2);
  } else {
    if (txn_codes && s->txn_cnt) memcpy(txn_codes, s->frag ? (const int8_t *)s->h_tr : s->h_codes, s->txn_cnt);
    if (trailers && s->frag && s->tr_sz) memcpy(trailers, s->h_tr + s->tr_base, s->tr_sz);
  }
  if (keep) st_rlx(s->held, true);
  else st_rlx(s->ticket, (int64_t)-1);
  return FDGPU_OK;
}

int fdgpu_poll(fdgpu_engine_t *e, int64_t ticket, int8_t *txn_codes, int blocking) {
  return poll_slot(e, ticket, txn_codes, blocking, false);
}

int fdgpu_poll_keep(fdgpu_engine_t *e, int64_t ticket, int8_t *txn_codes, int blocking) {
  return poll_slot(e, ticket, txn_codes, blocking, true);
}

int fdgpu_poll_frags(fdgpu_engine_t *e, int64_t ticket, int8_t *codes, uint8_t *trailers, int blocking) {
  return poll_slot(e, ticket, codes, blocking, false, trailers);
}

/* fdgpu_submit with the parse on the device: upload (DMA from a registered
   region, or staged), then on the slot's stream parse -> scan -> expand ->
   verify -> combine -> parse-failure codes -> trailer pack, and the codes and
   trailers back to pinned memory. */
int64_t fdgpu_submit_frags(fdgpu_engine_t *e, uint8_t const *arena, uint64_t arena_sz, fdgpu_frag_ex_t const *fx,
                           uint64_t n, uint64_t trailer_sz) {
  if (!e || (!arena && arena_sz) || (!fx && n)) { set_err("null argument"); return FDGPU_ERR_INVAL; }
  if (arena_sz > e->cfg.max_arena || n > e->cfg.max_txn) { set_err("batch exceeds engine limits"); return FDGPU_ERR_INVAL; }
  if (trailer_sz > (uint64_t)n * FDT_TXN_MAX_SZ_BYTES + 4) { set_err("trailer buffer larger than the frags' maximum"); return FDGPU_ERR_INVAL; }
  uint64_t bound = 0;
  for (uint64_t t = 0; t < n; t++) {
    const fdgpu_frag_ex_t &f = fx[t];
    if ((uint64_t)f.off + f.sz > arena_sz || (f.tr_off & 3u) || (uint64_t)f.tr_off + f.tr_cap > trailer_sz ||
        f.tr_cap > FDT_TXN_MAX_SZ_BYTES) {
      set_err("frag %llu: out of arena or trailer bounds", (unsigned long long)t);
      return FDGPU_ERR_INVAL;
    }
    bound += fdt_frag_sig_bound(f.sz);
  }
  if (bound > e->cfg.max_sig) { set_err("batch may exceed max_sig (%llu)", (unsigned long long)e->cfg.max_sig); return FDGPU_ERR_INVAL; }
  std::lock_guard<std::mutex> lk(e->ring_mu);
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  Slot *s = free_slot(e);
  if (!s) { set_err("all ring slots hold unpolled batches"); return FDGPU_ERR_FULL; }
  if (!slot_frag_bufs(*s, e->cfg, trailer_sz) || !slot_ws(*s, bound)) return FDGPU_ERR_DEVICE;
  /* the slack past the arena needs no zeroing here: every device reader of
     a frag batch masks the bytes past its payload (fdt_reader, msg_block),
     only their presence (FDGPU_ARENA_SLACK allocated) matters */
  if (region_covers(e, arena, arena_sz)) {
    if (arena_sz) HIPCHK(hipMemcpyAsync(s->d_arena, arena, arena_sz, hipMemcpyHostToDevice, s->stream), FDGPU_ERR_DEVICE);
  } else {
    const uint64_t up = stage_arena(e, s, arena, arena_sz);
    if (up == UINT64_MAX) return FDGPU_ERR_DEVICE;
    if (arena_sz > up)
      HIPCHK(hipMemcpyAsync(s->d_arena + up, s->h_arena + up, arena_sz - up, hipMemcpyHostToDevice, s->stream),
             FDGPU_ERR_DEVICE);
  }
  const uint64_t tr_base = (n + 63) & ~63ull;
  if (n) {
    memcpy(s->h_fx, fx, n * sizeof(fdgpu_frag_ex_t));
    HIPCHK(hipMemcpyAsync(s->d_fx, s->h_fx, n * sizeof(fdgpu_frag_ex_t), hipMemcpyHostToDevice, s->stream), FDGPU_ERR_DEVICE);
    HIPCHK(fdgpu_launch_frag_ring(s->d_arena, s->d_fx, (uint32_t)n, s->d_txn_out, s->d_txn_sz, s->d_txd, s->d_cnt,
                                  s->d_sig0, s->d_blocktot, s->d_n_sig, s->d_sigs, s->d_txns, s->stream),
           FDGPU_ERR_DEVICE);
    HIPCHK(fdgpu_launch_verify_sigs(s->d_arena, s->d_sigs, (uint32_t)bound, nullptr, e->d_btab, s->d_ws, s->d_sig_codes,
                                    ring_kflags(e, s, bound), s->stream, s->d_n_sig, e->resident_blocks, e->kc_seed),
           FDGPU_ERR_DEVICE);
    HIPCHK(fdgpu_launch_frag_finish(s->d_txns, (uint32_t)n, s->d_sig_codes, s->d_txn_sz, s->d_fx, s->d_txn_out,
                                    (int8_t *)s->d_tr, s->d_tr + tr_base, s->stream),
           FDGPU_ERR_DEVICE);
    HIPCHK(hipMemcpyAsync(s->h_tr, s->d_tr, tr_base + trailer_sz, hipMemcpyDeviceToHost, s->stream), FDGPU_ERR_DEVICE);
  }
  slot_flag_next(s);
  if (e->flag_poll && !e->drop_flag) HIPCHK(hipStreamWriteValue32(s->stream, s->d_flag, s->flag_seq, 0), FDGPU_ERR_DEVICE);
  HIPCHK(hipEventRecord(s->done, s->stream), FDGPU_ERR_DEVICE);
  s->staged = false;
  st_rlx(s->held, false);
  st_rlx(s->polls, 0u);
  s->frag = true;
  s->io = false;
  s->tr_sz = trailer_sz;
  s->tr_base = tr_base;
  st_rlx(s->ticket, e->next_ticket++);
  s->txn_cnt = n;
  return s->ticket;
}

uint32_t fdgpu_frag_out_cap(uint32_t sz) {
  return (uint32_t)(((uint64_t)sz + 1u) / 2u * 2u + fdgpu_frag_fp_bound(sz) + 2u);
}

/* Gathered frag batches (the header's fdgpu_submit_frags_io): the device
   reads each payload from its registered host region (the in dcache) into
   the slot arena -- and, for a frag naming an in link, re-reads the frag's
   mcache line afterwards (the overrun re-check) -- then parse -> expand ->
   verify -> finish on the slot's stream; the finish kernel writes the out
   frags into the registered out region and [codes][tags][out sizes] into the
   slot's pinned results, both in place, and the stream stores the completion
   word.  No copies are queued. */
}  // extern "C"

namespace {

/* the rest of a gathered batch after its verify: finish (out frags and
   results written over the bus), the completion word, the done event */
int io_tail(fdgpu_engine_t *e, Slot *s) {
  const uint64_t n = s->m_n, cb = s->m_cb;
  HIPCHK(fdgpu_launch_frag_finish_io(s->d_txns, (uint32_t)n, s->d_sig_codes, s->d_txn_sz, s->d_fxio, s->d_txn_out,
                                     s->m_arena, s->m_seed, s->m_out, (int8_t *)s->d_trh, (uint64_t *)(s->d_trh + cb),
                                     (uint16_t *)(s->d_trh + cb + n * 8), s->d_io_cnt, s->stream),
         FDGPU_ERR_DEVICE);
  s->io_cnt_dirty = false;
  slot_flag_next(s);
  if (e->flag_poll && !e->drop_flag) HIPCHK(hipStreamWriteValue32(s->stream, s->d_flag, s->flag_seq, 0), FDGPU_ERR_DEVICE);
  HIPCHK(hipEventRecord(s->done, s->stream), FDGPU_ERR_DEVICE);
  return FDGPU_OK;
}

bool merge_free(const fdgpu_engine_t *e, const Merge &m) {
  if (e->flag_poll) return __atomic_load_n(m.h_flag, __ATOMIC_ACQUIRE) == m.seq;
  return !m.seq || hipEventQuery(m.ev[(m.seq - 1) % e->merge_tabs]) == hipSuccess;
}

/* FDGPU_FLAG_MERGE (ring_mu held): the verifies of the batches waiting, as
   one launch on a merge stream that is idle -- or, forced (a blocking poll
   waits on one of them), on the next one anyway -- then each batch's tail on
   its own stream behind it */
int merge_kick_queue(fdgpu_engine_t *e, bool force);

/* a HIP error part-way leaves batches with tickets issued and nothing (or
   only part) queued for them: each is marked failed, so its poll returns
   the error instead of waiting for a completion word that never comes */
int merge_kick(fdgpu_engine_t *e, bool force) {
  const int rc = merge_kick_queue(e, force);
  if (rc) {
    for (Slot *s : e->pending) if (s->vpending) { s->vpending = false; s->failed = true; }
    e->pending.clear();
  }
  return rc;
}

int merge_kick_queue(fdgpu_engine_t *e, bool force) {
  if (e->pending.empty()) return FDGPU_OK;
  if (e->fail_merge_at && ++e->merge_calls == e->fail_merge_at) {
    set_err("injected merge failure (FDGPU_DEBUG_FAIL_MERGE)");
    return FDGPU_ERR_DEVICE;
  }
  const uint32_t nms = (uint32_t)e->merges.size();
  int mi = -1;
  for (uint32_t k = 0; k < nms && mi < 0; k++) {
    const uint32_t j = (e->merge_rr + k) % nms;
    if (merge_free(e, e->merges[j])) mi = (int)j;
  }
  if (mi < 0) {
    if (!force) return FDGPU_OK;
    mi = (int)(e->merge_rr % nms);
  }
  e->merge_rr = (uint32_t)mi + 1;
  Merge &m = e->merges[(size_t)mi];
  const uint32_t ti = m.seq % e->merge_tabs;
  const uint32_t nb = (uint32_t)e->pending.size();
  for (Slot *s : e->pending) HIPCHK(hipStreamWaitEvent(m.stream, s->parsed, 0), FDGPU_ERR_DEVICE);
  if (nb == 1) {                               /* alone: the ring path's kernels (FDGPU_FLAG_PAIR_AUTO applies) */
    Slot *s = e->pending[0];
    HIPCHK(fdgpu_launch_verify_sigs(s->m_arena, s->d_sigs, (uint32_t)s->m_bound, nullptr, e->d_btab, s->d_ws,
                                    s->d_sig_codes, ring_kflags(e, s, s->m_bound), m.stream, s->d_io_cnt,
                                    e->resident_blocks, e->kc_seed, 1),
           FDGPU_ERR_DEVICE);
  } else {
    fdgpu_mbatch_t *tab = m.h_tab + (size_t)ti * e->cfg.ring_depth;
    uint32_t grid_max = 0, slow_max = 0;
    for (uint32_t j = 0; j < nb; j++) {
      Slot *s = e->pending[j];
      const uint32_t grid = (uint32_t)((s->m_bound + FDGPU_BLOCK - 1) / FDGPU_BLOCK);
      uint32_t slow = grid < e->resident_blocks ? grid : e->resident_blocks;
      if (slow > FDGPU_FULL_BLOCKS) slow = FDGPU_FULL_BLOCKS;
      uint32_t *cnt = fdgpu_verify_cnt_word(s->d_ws, (uint32_t)s->m_bound);
      st_rlx(s->k_sigs, s->m_bound);
      st_rlx(s->k_lanes, s->m_bound);          /* one lane each: the merged launch never takes the pair kernel */
      tab[j] = fdgpu_mbatch_t{s->m_arena, s->d_sigs, s->d_io_cnt, s->d_ws, s->d_sig_codes,
                              cnt - (size_t)grid * FDGPU_BLOCK, cnt, (uint32_t)s->m_bound, slow};
      grid_max = grid > grid_max ? grid : grid_max;
      slow_max = slow > slow_max ? slow : slow_max;
    }
    HIPCHK(fdgpu_launch_verify_multi(m.d_tab + (size_t)ti * e->cfg.ring_depth, nb, grid_max, slow_max, e->d_btab,
                                     kflags(e) & ~(uint32_t)FDGPU_FLAG_KPAIR, m.stream),
           FDGPU_ERR_DEVICE);
  }
  HIPCHK(hipEventRecord(m.ev[ti], m.stream), FDGPU_ERR_DEVICE);
  ++m.seq;
  if (e->flag_poll) HIPCHK(hipStreamWriteValue32(m.stream, m.d_flag, m.seq, 0), FDGPU_ERR_DEVICE);
  for (Slot *s : e->pending) {
    HIPCHK(hipStreamWaitEvent(s->stream, m.ev[ti], 0), FDGPU_ERR_DEVICE);
    const int rc = io_tail(e, s);
    if (rc) return rc;
    s->vpending = false;
  }
  e->merge_launches++;
  e->merge_batches += nb;
  e->pending.clear();
  return FDGPU_OK;
}

}  // namespace

extern "C" {

int64_t fdgpu_submit_frags_io(fdgpu_engine_t *e, fdgpu_frag_io_t const *fio, uint64_t n, uint8_t *out,
                              uint64_t out_sz, uint64_t hash_seed, fdgpu_link_t const *links, uint64_t link_cnt) {
  const uint64_t sp0 = g_sp_on ? sp_now() : 0;
  if (!e || (!fio && n) || (!out && out_sz) || (!links && link_cnt)) { set_err("null argument"); return FDGPU_ERR_INVAL; }
  if (n > e->cfg.max_txn) { set_err("batch exceeds engine limits"); return FDGPU_ERR_INVAL; }
  if (link_cnt > FDGPU_LINK_MAX) { set_err("more than %lu links", (unsigned long)FDGPU_LINK_MAX); return FDGPU_ERR_INVAL; }
  std::lock_guard<std::mutex> lk(e->ring_mu);
  const fdgpu_engine::Reg *ro = out_sz ? region_of(e, (uintptr_t)out, out_sz) : nullptr;
  if (out_sz && !ro) { set_err("out range not inside a registered region"); return FDGPU_ERR_UNREG; }
  /* each named link's mcache: its device-side address (the lines are read
     in place over the bus) */
  uint64_t ldev[FDGPU_LINK_MAX], lmask[FDGPU_LINK_MAX];
  for (uint64_t l = 0; l < link_cnt; l++) {
    const uint64_t d = links[l].depth;
    if (!d || (d & (d - 1)) || (links[l].mcache & 7u)) {
      set_err("link %llu: bad depth or a misaligned mcache", (unsigned long long)l);
      return FDGPU_ERR_INVAL;
    }
    const fdgpu_engine::Reg *rm = region_of(e, (uintptr_t)links[l].mcache, d * 32u);
    if (!rm) {
      set_err("link %llu: mcache not inside a registered region", (unsigned long long)l);
      return FDGPU_ERR_UNREG;
    }
    ldev[l] = rm->dbase + (links[l].mcache - rm->base);
    lmask[l] = d - 1;
  }
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  Slot *s = free_slot(e);
  if (!s) { set_err("all ring slots hold unpolled batches"); return FDGPU_ERR_FULL; }
  /* results: codes (padded to 64) + 8 B tags + 2 B sizes, in the trailer buffer */
  const uint64_t cb = (n + 63) & ~63ull, res_sz = cb + n * 10;
  if (!slot_frag_bufs(*s, e->cfg, res_sz)) return FDGPU_ERR_DEVICE;
  /* the frag records, then (64-B aligned) the payload addresses, then the
     re-check pairs {line address, seq}, in pinned memory the gather reads in
     place */
  const uint64_t src_at = (n * sizeof(fdgpu_frag_ex_t) + 63) & ~63ull;
  const uint64_t chk_at = src_at + ((n * sizeof(uint64_t) + 63) & ~63ull);
  if (!slot_io_bufs(*s, e->cfg)) return FDGPU_ERR_DEVICE;
  static_assert(sizeof(fdgpu_frag_ex_t) == 16, "one 16-B streaming store per record");
  fdgpu_frag_ex_t *h_fx = (fdgpu_frag_ex_t *)s->h_io;
  uint64_t *h_src = (uint64_t *)(s->h_io + src_at);
  uint64_t *h_chk = (uint64_t *)(s->h_io + chk_at);
  /* bounds: every payload inside a registered region (16-B aligned: the
     gather reads 16-B units up to round16(sz), inside the payload's own
     64-B chunks), every out frag inside out, the packed arena within
     max_arena, the signature bound within max_sig, every named link given.

     DMA gather (FDGPU_IO_DMA=1, g_io_dma): the frags' payloads are grouped into
     ranges of source bytes -- per registered region, a run of this batch's
     frags with gaps of at most FDGPU_IO_GAP (a round robin's other tiles'
     frags lie between this tile's) -- and each range is copied into the
     slot's mirror by the DMA engines; the records then name a range and an
     offset in it, and the payloads are parsed and verified where the copy
     put them.  More than FDGPU_IO_RANGES_MAX ranges, or more bytes than the
     mirror holds: this batch takes the kernel-load path. */
  const uint64_t rtab_at = chk_at + ((n * 2 * sizeof(uint64_t) + 63) & ~63ull);
  uint64_t *h_rtab = (uint64_t *)(s->h_io + rtab_at);
  struct Range { uintptr_t lo, hi; };
  static thread_local Range rg[FDGPU_IO_RANGES_MAX];
  uint32_t nr = 0;
  uint64_t dev_off = 0, bound = 0;
  bool any_chk = false;
  bool dma = g_io_dma && s->d_mirror;
  constexpr uintptr_t FDGPU_IO_GAP = 4096;
  auto fill = [&](bool use_dma) -> int {           /* 0, 1: redo without DMA, < 0: error */
    const fdgpu_engine::Reg *rc = nullptr;
    const fdgpu_engine::Reg *open_reg[16];
    uint32_t open_rng[16], n_open = 0;
    nr = 0; dev_off = 0; bound = 0; any_chk = false;
    for (uint64_t t = 0; t < n; t++) {
      const fdgpu_frag_io_t &f = fio[t];
      const uint64_t q = ((uint64_t)f.sz + 15u) & ~15ull;
      if (f.sz > FDT_TXN_MTU_BYTES || (f.src & 15u) || (f.out_off & 1u) || (uint64_t)f.out_off + f.out_cap > out_sz ||
          f.out_cap > 0xFFFFu || f.link > link_cnt) {
        set_err("frag %llu: size, alignment, out bounds or link", (unsigned long long)t);
        return FDGPU_ERR_INVAL;
      }
      if (!rc || f.src < rc->base || f.src + q > rc->end) rc = region_of(e, (uintptr_t)f.src, q);
      if (!rc) { set_err("frag %llu: payload not inside a registered region", (unsigned long long)t); return FDGPU_ERR_UNREG; }
      uint32_t off, sz = f.sz;
      if (use_dma) {
        uint32_t k = 0;
        while (k < n_open && open_reg[k] != rc) k++;
        uint32_t ri = k < n_open ? open_rng[k] : UINT32_MAX;
        if (ri != UINT32_MAX && f.src >= rg[ri].lo && f.src <= rg[ri].hi + FDGPU_IO_GAP) {
          rg[ri].hi = std::max<uintptr_t>(rg[ri].hi, f.src + q);
        } else {
          if (nr == FDGPU_IO_RANGES_MAX || (k == n_open && n_open == 16)) return 1;
          ri = nr++;
          rg[ri] = Range{(uintptr_t)f.src, (uintptr_t)(f.src + q)};
          if (k == n_open) { open_reg[n_open] = rc; n_open++; }
          open_rng[k] = ri;
        }
        off = (uint32_t)(f.src - rg[ri].lo);
        sz |= ri << 16;
      } else {
        /* streaming stores: the records are for the device (read over the
           bus), not this core -- no line fills for them, nothing to snoop */
        _mm_stream_si64((long long *)&h_src[t], (long long)(rc->dbase + (f.src - rc->base)));
        off = (uint32_t)dev_off;
        dev_off += q;
        if (dev_off > e->cfg.max_arena) { set_err("frags exceed the engine's arena"); return FDGPU_ERR_INVAL; }
      }
      _mm_stream_si128((__m128i *)&h_fx[t], _mm_set_epi32((int)f.out_cap, (int)f.out_off, (int)sz, (int)off));
      if (f.link) {                                       /* {line address, seq}; fd_frag_meta_t.seq: offset 0 */
        _mm_stream_si128((__m128i *)&h_chk[2 * t],
                         _mm_set_epi64x((long long)f.seq, (long long)(ldev[f.link - 1] + (f.seq & lmask[f.link - 1]) * 32u)));
        any_chk = true;
      } else {
        _mm_stream_si64((long long *)&h_chk[2 * t], 0);
      }
      bound += fdt_frag_sig_bound(f.sz);
    }
    if (use_dma) {                                     /* each range's place in the mirror */
      uint64_t m = 0;
      for (uint32_t r = 0; r < nr; r++) {
        h_rtab[r] = m;
        m = (m + (rg[r].hi - rg[r].lo) + 63u) & ~63ull;
      }
      if (m > s->mirror_cap) return 1;
    }
    return 0;
  };
  int frc = fill(dma);
  if (frc == 1) { dma = false; frc = fill(false); }
  if (frc < 0) return frc;
  _mm_sfence();                                        /* the streamed records reach memory before the launches */
  if (bound > e->cfg.max_sig) { set_err("batch may exceed max_sig (%llu)", (unsigned long long)e->cfg.max_sig); return FDGPU_ERR_INVAL; }
  const uint64_t sp1 = g_sp_on ? sp_now() : 0;
  if (!slot_ws(*s, bound)) return FDGPU_ERR_DEVICE;
  /* four kernels: ingest (gather, re-check of the in mcache lines, parse
     and expand; it keeps the records on the device and zeroes the verify
     queue counter), verify and its fallback, finish -- the out frags and
     the results written in place over the bus -- then the completion word */
  uint8_t *out_dev = out_sz ? (uint8_t *)(ro->dbase + ((uintptr_t)out - ro->base)) : nullptr;
  uint8_t *arena = dma ? s->d_mirror : s->d_arena;
  if (n) {
    const fdgpu_frag_ex_t *d_fx = s->d_fxio;
    const bool zero_cnt = !(kflags(e) & FDGPU_FLAG_KCACHE);
    for (uint32_t r = 0; dma && r < nr; r++)
      HIPCHK(hipMemcpyAsync(s->d_mirror + h_rtab[r], (const void *)rg[r].lo, rg[r].hi - rg[r].lo, hipMemcpyHostToDevice,
                            s->stream),
             FDGPU_ERR_DEVICE);
    if (s->io_cnt_dirty) HIPCHK(hipMemsetAsync(s->d_io_cnt, 0, 64, s->stream), FDGPU_ERR_DEVICE);
    s->io_cnt_dirty = false;
    HIPCHK(fdgpu_launch_frag_ingest_io((const uint64_t *)(s->d_ioh + src_at), (const fdgpu_frag_ex_t *)s->d_ioh,
                                       any_chk ? (const uint64_t *)(s->d_ioh + chk_at) : nullptr,
                                       dma ? (const uint64_t *)(s->d_ioh + rtab_at) : nullptr, (uint32_t)n,
                                       arena, s->d_fxio, s->d_txn_out, s->d_txn_sz, s->d_sigs, s->d_txns,
                                       s->d_io_cnt,
                                       zero_cnt ? fdgpu_verify_cnt_word(s->d_ws, (uint32_t)bound) : nullptr, s->stream),
           FDGPU_ERR_DEVICE);
    s->io_cnt_dirty = true;                            /* until this batch's finish is queued */
    if (!e->merges.empty() && zero_cnt && bound) {
      /* the verify waits to be merged with the other batches ready (merge_kick) */
      HIPCHK(hipEventRecord(s->parsed, s->stream), FDGPU_ERR_DEVICE);
      s->vpending = true;
      s->m_n = (uint32_t)n; s->m_seed = hash_seed; s->m_out = out_dev; s->m_cb = cb; s->m_bound = bound;
      s->m_arena = arena;
      e->pending.push_back(s);
      s->staged = false; st_rlx(s->held, false); st_rlx(s->polls, 0u); s->frag = true; s->io = true; s->tr_sz = 0; s->tr_base = 0;
      st_rlx(s->ticket, e->next_ticket++);
      s->txn_cnt = n;
      /* a failed merge marks this batch failed: its poll reports the error
         (returning the error here would leave the slot's ticket unknown to the
         caller, and the slot occupied for good) */
      (void)merge_kick(e, false);
      return s->ticket;
    }
    HIPCHK(fdgpu_launch_verify_sigs(arena, s->d_sigs, (uint32_t)bound, nullptr, e->d_btab, s->d_ws, s->d_sig_codes,
                                    ring_kflags(e, s, bound), s->stream, s->d_io_cnt, e->resident_blocks, e->kc_seed,
                                    zero_cnt),
           FDGPU_ERR_DEVICE);
    HIPCHK(fdgpu_launch_frag_finish_io(s->d_txns, (uint32_t)n, s->d_sig_codes, s->d_txn_sz, d_fx, s->d_txn_out,
                                       arena, hash_seed, out_dev, (int8_t *)s->d_trh, (uint64_t *)(s->d_trh + cb),
                                       (uint16_t *)(s->d_trh + cb + n * 8), s->d_io_cnt, s->stream),
           FDGPU_ERR_DEVICE);
    s->io_cnt_dirty = false;
  }
  slot_flag_next(s);
  if (e->flag_poll && !e->drop_flag) HIPCHK(hipStreamWriteValue32(s->stream, s->d_flag, s->flag_seq, 0), FDGPU_ERR_DEVICE);
  HIPCHK(hipEventRecord(s->done, s->stream), FDGPU_ERR_DEVICE);
  s->staged = false;
  st_rlx(s->held, false);
  st_rlx(s->polls, 0u);
  s->frag = true;
  s->io = true;
  s->tr_sz = 0;
  s->tr_base = 0;
  st_rlx(s->ticket, e->next_ticket++);
  s->txn_cnt = n;
  if (g_sp_on) {
    const uint64_t sp2 = sp_now();
    g_sp_loop += sp1 - sp0; g_sp_enq += sp2 - sp1; g_sp_calls++; g_sp_frags += n;
  }
  return s->ticket;
}

int fdgpu_poll_frags_io(fdgpu_engine_t *e, int64_t ticket, int8_t *codes, uint64_t *tags, uint16_t *out_szs,
                        int blocking) {
  return poll_slot(e, ticket, codes, blocking, false, nullptr, tags, out_szs);
}

int fdgpu_stage_cancel(fdgpu_engine_t *e) {
  if (!e) return FDGPU_ERR_INVAL;
  std::lock_guard<std::mutex> lk(e->ring_mu);
  for (auto &c : e->slots) if (c.staged) { c.staged = false; return FDGPU_OK; }
  return FDGPU_ERR_INVAL;
}

int fdgpu_release(fdgpu_engine_t *e, int64_t ticket) {
  if (!e) return FDGPU_ERR_INVAL;
  std::lock_guard<std::mutex> lk(e->ring_mu);
  for (auto &c : e->slots)
    if (c.ticket == ticket && ticket >= 0 && c.held) { st_rlx(c.held, false); st_rlx(c.ticket, (int64_t)-1); return FDGPU_OK; }
  set_err("ticket %lld not held", (long long)ticket);
  return FDGPU_ERR_TICKET;
}

int fdgpu_host_register(fdgpu_engine_t *e, void *p, uint64_t sz) {
  if (!e || !p || !sz) { set_err("null argument"); return FDGPU_ERR_INVAL; }
  const uintptr_t a = (uintptr_t)p & ~(uintptr_t)4095, b = ((uintptr_t)p + sz + 4095) & ~(uintptr_t)4095;
  std::lock_guard<std::mutex> lk(e->ring_mu);
  std::lock_guard<std::mutex> rk(g_reg_mu);
  /* a range inside a region already pinned (by any engine) shares it;
     a range that only partly overlaps one cannot be pinned */
  auto it = g_regions.upper_bound(a);
  uintptr_t base = 0, end = 0, dbase = 0;
  if (it != g_regions.begin()) {
    auto pv = std::prev(it);
    if (pv->first <= a && pv->second.end >= b) {
      base = pv->first; end = pv->second.end; dbase = pv->second.dbase; pv->second.refs++;
    } else if (pv->second.end > a) {
      set_err("range partly overlaps a registered region");
      return FDGPU_ERR_INVAL;
    }
  }
  if (!base) {
    if (it != g_regions.end() && it->first < b) { set_err("range partly overlaps a registered region"); return FDGPU_ERR_INVAL; }
    HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
    HIPCHK(hipHostRegister((void *)a, b - a, hipHostRegisterPortable | hipHostRegisterMapped), FDGPU_ERR_DEVICE);
    void *dp = nullptr;
    if (hipHostGetDevicePointer(&dp, (void *)a, 0) != hipSuccess || !dp) {
      (void)hipGetLastError();
      (void)hipHostUnregister((void *)a);
      set_err("registered region has no device address");
      return FDGPU_ERR_DEVICE;
    }
    g_regions[a] = {b, 1, (uintptr_t)dp};
    base = a; end = b; dbase = (uintptr_t)dp;
  }
  e->regions.push_back({a, base, end, dbase});
  return FDGPU_OK;
}

int fdgpu_host_unregister(fdgpu_engine_t *e, void *p) {
  if (!e || !p) return FDGPU_ERR_INVAL;
  const uintptr_t a = (uintptr_t)p & ~(uintptr_t)4095;
  std::lock_guard<std::mutex> lk(e->ring_mu);
  for (size_t i = e->regions.size(); i-- > 0;) {            /* the latest registration of this range */
    if (e->regions[i].user != a) continue;
    for (auto &sl : e->slots) if (sl.stream) (void)hipStreamSynchronize(sl.stream);   /* no DMA still reads it */
    region_release(e->device, e->regions[i].base);
    e->regions.erase(e->regions.begin() + (long)i);
    return FDGPU_OK;
  }
  set_err("region not registered with this engine");
  return FDGPU_ERR_INVAL;
}

int fdgpu_verify_device(fdgpu_engine_t *e, void const *d_arena, void const *d_sig_desc, uint64_t sig_cnt,
                        void const *d_txn_desc, uint64_t txn_cnt, int8_t *d_sig_codes, int8_t *d_txn_codes,
                        void *hip_stream) {
  if (!e || sig_cnt > 0xFFFFFFF0ull || txn_cnt > 0xFFFFFFF0ull) return FDGPU_ERR_INVAL;
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : e->compute;
  if (!d_sig_codes) {
    if (e->scratch_cap < sig_cnt + 16) {
      if (e->d_scratch_codes) { HIPCHK(hipStreamSynchronize(st), FDGPU_ERR_DEVICE); (void)hipFree(e->d_scratch_codes); }
      e->d_scratch_codes = nullptr;
      HIPCHK(hipMalloc((void **)&e->d_scratch_codes, sig_cnt + 16), FDGPU_ERR_DEVICE);
      e->scratch_cap = sig_cnt + 16;
    }
    d_sig_codes = e->d_scratch_codes;
  }
  return enqueue_verify(e, (const uint8_t *)d_arena, (const fdgpu_sig_desc_t *)d_sig_desc, nullptr, sig_cnt,
                        (const fdgpu_txn_desc_t *)d_txn_desc, txn_cnt, d_sig_codes, d_txn_codes, st);
}

/* ----------------------------------------------- device-resident batches */

}  // extern "C"

struct fdgpu_dev_batch {
  uint8_t *d_arena = nullptr;
  fdgpu_sig_desc_t *d_sigs = nullptr;
  uint32_t *d_perm = nullptr;               /* NULL: descriptors in transaction order */
  fdgpu_txn_desc_t *d_txns = nullptr;
  int8_t *d_sig_codes = nullptr, *d_txn_codes = nullptr;
  uint64_t n_sig = 0, n_txn = 0;
  /* fdgpu_dev_batch_own_queue: a private stream + workspace, so verifies of
     different batches run concurrently (the next batch's waves fill the CUs
     the previous one's last, partial round leaves idle) */
  hipStream_t stream = nullptr;
  uint32_t *d_ws = nullptr;
  /* frag batches (GPU-side ingest): raw payloads in d_arena; the descriptors
     above are produced on the device by each verify, n_sig is the bound the
     buffers and the grid are sized for until a codes() call reads the count */
  bool frags = false;
  int device = 0;
  hipStream_t compute = nullptr;            /* the engine's stream (the batch's queue until own_queue) */
  fdgpu_frag_t *d_frags = nullptr;
  uint8_t *d_txn_out = nullptr;
  uint16_t *d_txn_sz = nullptr;
  fdgpu_txn_t *d_txd = nullptr;
  uint32_t *d_cnt = nullptr, *d_sig0 = nullptr, *d_blocktot = nullptr, *d_n_sig = nullptr;
  uint64_t n_sig_bound = 0;
};

namespace {
hipStream_t batch_stream(fdgpu_engine_t *e, fdgpu_dev_batch_t *b) { return b->stream ? b->stream : e->compute; }
uint32_t *batch_ws(fdgpu_engine_t *e, fdgpu_dev_batch_t *b) { return b->d_ws ? b->d_ws : e->d_ws; }
}  // namespace

extern "C" {

uint64_t fdgpu_dev_batch_sig_cnt(fdgpu_dev_batch_t const *b) {
  if (!b) return 0;
  if (!b->frags) return b->n_sig;
  uint32_t n = 0;                             /* the count the last verify produced on the device */
  if (hipSetDevice(b->device) != hipSuccess) return 0;
  if (hipStreamSynchronize(b->stream ? b->stream : b->compute) != hipSuccess) return 0;
  if (hipMemcpy(&n, b->d_n_sig, sizeof(n), hipMemcpyDeviceToHost) != hipSuccess) return 0;
  return n;
}

int fdgpu_dev_batch_device_ptrs(fdgpu_dev_batch_t const *b, void **d_arena, void **d_sig_desc, void **d_perm,
                                void **d_txn_desc, int8_t **d_sig_codes, int8_t **d_txn_codes) {
  if (!b) return FDGPU_ERR_INVAL;
  if (d_arena) *d_arena = b->d_arena;
  if (d_sig_desc) *d_sig_desc = b->d_sigs;
  if (d_perm) *d_perm = b->d_perm;
  if (d_txn_desc) *d_txn_desc = b->d_txns;
  if (d_sig_codes) *d_sig_codes = b->d_sig_codes;
  if (d_txn_codes) *d_txn_codes = b->d_txn_codes;
  return FDGPU_OK;
}

int fdgpu_dev_batch_own_queue(fdgpu_engine_t *e, fdgpu_dev_batch_t *b) {
  if (!e || !b) return FDGPU_ERR_INVAL;
  if (b->stream) return FDGPU_OK;
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  const uint64_t nsig = b->frags ? b->n_sig_bound : b->n_sig;
  if (hipMalloc((void **)&b->d_ws, fdgpu_ws_bytes(nsig ? nsig : 1)) != hipSuccess) {
    b->d_ws = nullptr; set_err("batch workspace alloc"); return FDGPU_ERR_DEVICE;
  }
  if (hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) != hipSuccess) {
    (void)hipFree(b->d_ws); b->d_ws = nullptr; b->stream = nullptr; set_err("batch stream"); return FDGPU_ERR_DEVICE;
  }
  e->batch_streams.push_back(b->stream);
  return FDGPU_OK;
}

void fdgpu_dev_batch_free(fdgpu_engine_t *e, fdgpu_dev_batch_t *b) {
  if (!b) return;
  if (e) { (void)hipSetDevice(e->device); (void)hipStreamSynchronize(e->compute); }
  if (b->stream) {
    (void)hipStreamSynchronize(b->stream);
    if (e) {
      auto &v = e->batch_streams;
      for (size_t i = 0; i < v.size(); i++) if (v[i] == b->stream) { v.erase(v.begin() + (long)i); break; }
    }
    (void)hipStreamDestroy(b->stream);
  }
  if (b->d_ws) (void)hipFree(b->d_ws);
  if (b->d_arena) (void)hipFree(b->d_arena);
  if (b->d_sigs) (void)hipFree(b->d_sigs);
  if (b->d_perm) (void)hipFree(b->d_perm);
  if (b->d_txns) (void)hipFree(b->d_txns);
  if (b->d_sig_codes) (void)hipFree(b->d_sig_codes);
  if (b->d_txn_codes) (void)hipFree(b->d_txn_codes);
  for (void *p : {(void *)b->d_frags, (void *)b->d_txn_out, (void *)b->d_txn_sz, (void *)b->d_txd, (void *)b->d_cnt,
                  (void *)b->d_sig0, (void *)b->d_blocktot, (void *)b->d_n_sig})
    if (p) (void)hipFree(p);
  delete b;
}

fdgpu_dev_batch_t *fdgpu_dev_batch_upload(fdgpu_engine_t *e, uint8_t const *arena, uint64_t arena_sz,
                                          fdgpu_txn_t const *txns, uint64_t txn_cnt) {
  if (!e || (!arena && arena_sz) || (!txns && txn_cnt)) { set_err("null argument"); return nullptr; }
  if (arena_sz > 0xFFFFFFF0ull || txn_cnt > 0xFFFFFFF0ull) { set_err("batch exceeds 32-bit offsets"); return nullptr; }
  HIPCHK(hipSetDevice(e->device), nullptr);
  uint64_t total = 0;
  for (uint64_t t = 0; t < txn_cnt; t++) total += (txns[t].sig_cnt >= 1 && txns[t].sig_cnt <= 16) ? txns[t].sig_cnt : 0;
  std::vector<fdgpu_sig_desc_t> sd(total + 1);
  std::vector<fdgpu_txn_desc_t> td(txn_cnt + 1);
  std::vector<uint32_t> pm(bucket(e) ? total + 1 : 0);
  const int64_t ns = expand(arena_sz, txns, txn_cnt, total, sd.data(), td.data(), bucket(e) ? pm.data() : nullptr);
  if (ns < 0) return nullptr;
  fdgpu_dev_batch *b = new fdgpu_dev_batch();
  b->n_sig = (uint64_t)ns; b->n_txn = txn_cnt;
  auto fail = [&](const char *what) -> fdgpu_dev_batch_t * { set_err("%s", what); fdgpu_dev_batch_free(e, b); return nullptr; };
  if (hipMalloc((void **)&b->d_arena, arena_sz + FDGPU_ARENA_SLACK) != hipSuccess) return fail("arena alloc");
  if (hipMalloc((void **)&b->d_sigs, (ns + 1) * sizeof(fdgpu_sig_desc_t)) != hipSuccess) return fail("sig alloc");
  if (hipMalloc((void **)&b->d_txns, (txn_cnt + 1) * sizeof(fdgpu_txn_desc_t)) != hipSuccess) return fail("txn alloc");
  if (hipMalloc((void **)&b->d_sig_codes, ns + 16) != hipSuccess) return fail("code alloc");
  if (hipMalloc((void **)&b->d_txn_codes, txn_cnt + 16) != hipSuccess) return fail("code alloc");
  if (hipMemset(b->d_arena, 0, arena_sz + FDGPU_ARENA_SLACK) != hipSuccess) return fail("memset");
  if (arena_sz && hipMemcpy(b->d_arena, arena, arena_sz, hipMemcpyHostToDevice) != hipSuccess) return fail("h2d");
  if (ns && hipMemcpy(b->d_sigs, sd.data(), ns * sizeof(fdgpu_sig_desc_t), hipMemcpyHostToDevice) != hipSuccess) return fail("h2d");
  if (ns && !pm.empty()) {
    if (hipMalloc((void **)&b->d_perm, ns * sizeof(uint32_t)) != hipSuccess) return fail("perm alloc");
    if (hipMemcpy(b->d_perm, pm.data(), ns * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) return fail("h2d");
  }
  if (txn_cnt && hipMemcpy(b->d_txns, td.data(), txn_cnt * sizeof(fdgpu_txn_desc_t), hipMemcpyHostToDevice) != hipSuccess) return fail("h2d");
  if ((uint64_t)ns > e->ws_sig) {
    if (hipStreamSynchronize(e->compute) != hipSuccess) return fail("sync");
    if (ensure_ws(e, (uint64_t)ns) != FDGPU_OK) { fdgpu_dev_batch_free(e, b); return nullptr; }
  }
  return b;
}

fdgpu_dev_batch_t *fdgpu_dev_batch_upload_frags(fdgpu_engine_t *e, uint8_t const *arena, uint64_t arena_sz,
                                                fdgpu_frag_t const *frags, uint64_t frag_cnt) {
  if (!e || (!arena && arena_sz) || (!frags && frag_cnt)) { set_err("null argument"); return nullptr; }
  if (arena_sz > 0xFFFFFFF0ull || frag_cnt > 0x0FFFFFFFull) { set_err("batch exceeds 32-bit offsets"); return nullptr; }
  uint64_t bound = 0;
  for (uint64_t t = 0; t < frag_cnt; t++) {
    if ((uint64_t)frags[t].off + frags[t].sz > arena_sz) {
      set_err("frag %llu out of arena bounds", (unsigned long long)t);
      return nullptr;
    }
    bound += fdgpu_frag_sig_bound(frags[t].sz);
  }
  HIPCHK(hipSetDevice(e->device), nullptr);
  fdgpu_dev_batch *b = new fdgpu_dev_batch();
  b->frags = true;
  b->device = e->device;
  b->compute = e->compute;
  b->n_txn = frag_cnt;
  b->n_sig = bound;
  b->n_sig_bound = bound;
  auto fail = [&](const char *what) -> fdgpu_dev_batch_t * { set_err("%s", what); fdgpu_dev_batch_free(e, b); return nullptr; };
  const uint64_t nt = frag_cnt + 1, nb = (frag_cnt + 1023) / 1024 + 1;
  if (hipMalloc((void **)&b->d_arena, arena_sz + FDGPU_ARENA_SLACK) != hipSuccess) return fail("arena alloc");
  if (hipMalloc((void **)&b->d_frags, nt * sizeof(fdgpu_frag_t)) != hipSuccess) return fail("frag alloc");
  if (hipMalloc((void **)&b->d_txn_out, nt * 852u) != hipSuccess) return fail("txn alloc");
  if (hipMalloc((void **)&b->d_txn_sz, nt * sizeof(uint16_t)) != hipSuccess) return fail("txn alloc");
  if (hipMalloc((void **)&b->d_txd, nt * sizeof(fdgpu_txn_t)) != hipSuccess) return fail("txn alloc");
  if (hipMalloc((void **)&b->d_cnt, nt * sizeof(uint32_t)) != hipSuccess) return fail("scan alloc");
  if (hipMalloc((void **)&b->d_sig0, nt * sizeof(uint32_t)) != hipSuccess) return fail("scan alloc");
  if (hipMalloc((void **)&b->d_blocktot, nb * sizeof(uint32_t)) != hipSuccess) return fail("scan alloc");
  if (hipMalloc((void **)&b->d_n_sig, sizeof(uint32_t)) != hipSuccess) return fail("scan alloc");
  if (hipMalloc((void **)&b->d_sigs, (bound + 1) * sizeof(fdgpu_sig_desc_t)) != hipSuccess) return fail("sig alloc");
  if (hipMalloc((void **)&b->d_txns, nt * sizeof(fdgpu_txn_desc_t)) != hipSuccess) return fail("txn alloc");
  if (hipMalloc((void **)&b->d_sig_codes, bound + 16) != hipSuccess) return fail("code alloc");
  if (hipMalloc((void **)&b->d_txn_codes, frag_cnt + 16) != hipSuccess) return fail("code alloc");
  if (hipMemset(b->d_arena, 0, arena_sz + FDGPU_ARENA_SLACK) != hipSuccess) return fail("memset");
  if (hipMemset(b->d_n_sig, 0, sizeof(uint32_t)) != hipSuccess) return fail("memset");
  if (arena_sz && hipMemcpy(b->d_arena, arena, arena_sz, hipMemcpyHostToDevice) != hipSuccess) return fail("h2d");
  if (frag_cnt && hipMemcpy(b->d_frags, frags, frag_cnt * sizeof(fdgpu_frag_t), hipMemcpyHostToDevice) != hipSuccess)
    return fail("h2d");
  if (bound > e->ws_sig) {
    if (hipStreamSynchronize(e->compute) != hipSuccess) return fail("sync");
    if (ensure_ws(e, bound) != FDGPU_OK) { fdgpu_dev_batch_free(e, b); return nullptr; }
  }
  return b;
}

/* the ingest kernels of a frag batch (parse -> scan -> expand) on st */
static int enqueue_ingest(fdgpu_dev_batch_t *b, hipStream_t st) {
  HIPCHK(fdgpu_launch_frag_ingest(b->d_arena, b->d_frags, 2u, (uint32_t)b->n_txn, b->d_txn_out, b->d_txn_sz, b->d_txd,
                                  b->d_cnt, b->d_sig0, b->d_blocktot, b->d_n_sig, b->d_sigs, b->d_txns, st),
         FDGPU_ERR_DEVICE);
  return FDGPU_OK;
}

int fdgpu_dev_batch_verify(fdgpu_engine_t *e, fdgpu_dev_batch_t *b) {
  if (!e || !b) return FDGPU_ERR_INVAL;
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  if (!b->frags)
    return enqueue_verify(e, b->d_arena, b->d_sigs, b->d_perm, b->n_sig, b->d_txns, b->n_txn, b->d_sig_codes,
                          b->d_txn_codes, batch_stream(e, b), b->d_ws);
  const hipStream_t st = batch_stream(e, b);
  int rc = enqueue_ingest(b, st);
  if (rc) return rc;
  HIPCHK(fdgpu_launch_verify_sigs(b->d_arena, b->d_sigs, (uint32_t)b->n_sig_bound, nullptr, e->d_btab, batch_ws(e, b),
                                  b->d_sig_codes, kflags(e), st, b->d_n_sig, e->resident_blocks, e->kc_seed),
         FDGPU_ERR_DEVICE);
  HIPCHK(fdgpu_launch_combine(b->d_txns, (uint32_t)b->n_txn, b->d_sig_codes, b->d_txn_codes, nullptr, st),
         FDGPU_ERR_DEVICE);
  HIPCHK(fdgpu_launch_frag_codes(b->d_txn_sz, (uint32_t)b->n_txn, b->d_txn_codes, st), FDGPU_ERR_DEVICE);
  return FDGPU_OK;
}

int fdgpu_dev_batch_txns(fdgpu_engine_t *e, fdgpu_dev_batch_t *b, void *txn_out, uint16_t *txn_sz) {
  if (!e || !b || !b->frags) return FDGPU_ERR_INVAL;
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  HIPCHK(hipStreamSynchronize(batch_stream(e, b)), FDGPU_ERR_DEVICE);
  if (txn_out && b->n_txn) HIPCHK(hipMemcpy(txn_out, b->d_txn_out, b->n_txn * 852u, hipMemcpyDeviceToHost), FDGPU_ERR_DEVICE);
  if (txn_sz && b->n_txn)
    HIPCHK(hipMemcpy(txn_sz, b->d_txn_sz, b->n_txn * sizeof(uint16_t), hipMemcpyDeviceToHost), FDGPU_ERR_DEVICE);
  return FDGPU_OK;
}

int fdgpu_dev_batch_codes(fdgpu_engine_t *e, fdgpu_dev_batch_t *b, int8_t *txn_codes, int8_t *sig_codes) {
  if (!e || !b) return FDGPU_ERR_INVAL;
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  HIPCHK(hipStreamSynchronize(batch_stream(e, b)), FDGPU_ERR_DEVICE);
  if (b->frags) {                             /* the signature count the verify produced on the device */
    uint32_t n = 0;
    HIPCHK(hipMemcpy(&n, b->d_n_sig, sizeof(n), hipMemcpyDeviceToHost), FDGPU_ERR_DEVICE);
    b->n_sig = n;
  }
  if (txn_codes && b->n_txn) HIPCHK(hipMemcpy(txn_codes, b->d_txn_codes, b->n_txn, hipMemcpyDeviceToHost), FDGPU_ERR_DEVICE);
  if (sig_codes && b->n_sig) HIPCHK(hipMemcpy(sig_codes, b->d_sig_codes, b->n_sig, hipMemcpyDeviceToHost), FDGPU_ERR_DEVICE);
  return FDGPU_OK;
}

int fdgpu_dev_batch_time2(fdgpu_engine_t *e, fdgpu_dev_batch_t *b, int iters, double *wall_ms, double *ingest_ms,
                          double *verify_kernel_ms, double *combine_kernel_ms) {
  if (!e || !b || iters < 1) return FDGPU_ERR_INVAL;
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  const uint32_t flags = kflags(e);
  const hipStream_t st = batch_stream(e, b);
  const uint64_t nsig = b->frags ? b->n_sig_bound : b->n_sig;
  if (!b->d_ws && nsig > e->ws_sig) {
    HIPCHK(hipStreamSynchronize(e->compute), FDGPU_ERR_DEVICE);
    const int wrc = ensure_ws(e, nsig);
    if (wrc) return wrc;
  }
  std::vector<hipEvent_t> ev(4 * (size_t)iters + 1);
  for (auto &x : ev) HIPCHK(hipEventCreate(&x), FDGPU_ERR_DEVICE);
  int rc = FDGPU_OK;
  for (int i = 0; i < iters && rc == FDGPU_OK; i++) {
    if (hipEventRecord(ev[4 * i], st) != hipSuccess) rc = FDGPU_ERR_DEVICE;
    if (b->frags && rc == FDGPU_OK) rc = enqueue_ingest(b, st);
    if (hipEventRecord(ev[4 * i + 1], st) != hipSuccess) rc = FDGPU_ERR_DEVICE;
    if (fdgpu_launch_verify_sigs(b->d_arena, b->d_sigs, (uint32_t)nsig, b->d_perm, e->d_btab, batch_ws(e, b),
                                 b->d_sig_codes, flags, st, b->frags ? b->d_n_sig : nullptr, e->resident_blocks,
                                 e->kc_seed) != hipSuccess)
      rc = FDGPU_ERR_DEVICE;
    if (hipEventRecord(ev[4 * i + 2], st) != hipSuccess) rc = FDGPU_ERR_DEVICE;
    if (fdgpu_launch_combine(b->d_txns, (uint32_t)b->n_txn, b->d_sig_codes, b->d_txn_codes, nullptr, st) != hipSuccess)
      rc = FDGPU_ERR_DEVICE;
    if (b->frags && fdgpu_launch_frag_codes(b->d_txn_sz, (uint32_t)b->n_txn, b->d_txn_codes, st) != hipSuccess)
      rc = FDGPU_ERR_DEVICE;
    if (hipEventRecord(ev[4 * i + 3], st) != hipSuccess) rc = FDGPU_ERR_DEVICE;
  }
  if (rc == FDGPU_OK && hipEventSynchronize(ev[4 * (iters - 1) + 3]) != hipSuccess) rc = FDGPU_ERR_DEVICE;
  double si = 0, sv = 0, sc = 0;
  float ms = 0;
  for (int i = 0; rc == FDGPU_OK && i < iters; i++) {
    (void)hipEventElapsedTime(&ms, ev[4 * i], ev[4 * i + 1]); si += ms;
    (void)hipEventElapsedTime(&ms, ev[4 * i + 1], ev[4 * i + 2]); sv += ms;
    (void)hipEventElapsedTime(&ms, ev[4 * i + 2], ev[4 * i + 3]); sc += ms;
  }
  if (rc == FDGPU_OK) {
    (void)hipEventElapsedTime(&ms, ev[0], ev[4 * (iters - 1) + 3]);
    if (wall_ms) *wall_ms = ms;
    if (ingest_ms) *ingest_ms = b->frags ? si / iters : 0.0;
    if (verify_kernel_ms) *verify_kernel_ms = sv / iters;
    if (combine_kernel_ms) *combine_kernel_ms = sc / iters;
  } else {
    set_err("timing launch failed");
  }
  for (auto &x : ev) (void)hipEventDestroy(x);
  return rc;
}

/* for a frag batch the ingest kernels count in *verify_kernel_ms */
int fdgpu_dev_batch_time(fdgpu_engine_t *e, fdgpu_dev_batch_t *b, int iters, double *wall_ms, double *verify_kernel_ms,
                         double *combine_kernel_ms) {
  double ig = 0, v = 0;
  const int rc = fdgpu_dev_batch_time2(e, b, iters, wall_ms, &ig, &v, combine_kernel_ms);
  if (rc == FDGPU_OK && verify_kernel_ms) *verify_kernel_ms = v + ig;
  return rc;
}

int fdgpu_sync(fdgpu_engine_t *e) {
  if (!e) return FDGPU_ERR_INVAL;
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  HIPCHK(hipStreamSynchronize(e->compute), FDGPU_ERR_DEVICE);
  for (auto &s : e->slots) HIPCHK(hipStreamSynchronize(s.stream), FDGPU_ERR_DEVICE);
  for (auto st : e->batch_streams) HIPCHK(hipStreamSynchronize(st), FDGPU_ERR_DEVICE);
  return FDGPU_OK;
}

/* ------------------------------------------------------------ sync API */

/* The reference's synchronous per-call API (fd_ed25519.h:96-101,124-130) on
   one process-wide engine on device 0.  A call is one GPU round trip: about
   a millisecond, the lifetime of the verify kernel's single wave, not the
   CPU's ~30 us (bench.py `sync_*` lines).

   Calls from concurrent threads are coalesced (group commit): a caller that
   finds no batch in flight becomes the leader, takes every call queued so
   far as one batch (one txn per call) and verifies it; calls arriving
   meanwhile queue for the next leader.  A lone caller pays one round trip,
   N concurrent callers share theirs, so throughput grows with the number of
   callers instead of serialising on a lock.  The caller's current HIP device
   is saved and restored.

   A call whose message does not fit one batch arena (32-bit offsets: about
   2 GB) is verified alone: its k = SHA-512(R || A || M) is hashed on the
   device in arena-sized pieces of M (fdgpu_sha512_stream_kernel), then the
   verify runs from those digests -- the reference hashes any msg_sz
   (fd_ed25519_user.c:205-207), so size is never an error here.
   FDGPU_SYNC_ARENA_MAX=<bytes> lowers that limit (tests reach the path with
   small messages).

   The reference API has no error channel besides the verify codes, and it
   never answers a good signature with an error.  So an engine failure (no
   device, a HIP error) aborts the process by default, with the reason on stderr: a transient GPU fault must
   not turn valid transactions or blocks into rejected ones (replay's
   fd_executor_txn_verify, the shred FEC-root checks).  A caller that prefers
   to reject instead sets FDGPU_SYNC_FAIL_CLOSED=1: every call of the failed
   batch then returns FD_ED25519_ERR_SIG and fdgpu_sync_errors() counts the
   event (fdgpu_last_error() of the failing thread says why).
   FDGPU_SYNC_DEVICE=<n> puts the engine on device n (default 0). */
}  // extern "C"

namespace {

struct SyncReq {
  const uint8_t *msg, *sigs, *pubs;
  uint64_t msg_sz;
  uint32_t n;
  int code = 0;
  bool done = false;
};

struct SyncState {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<SyncReq *> pending;
  bool leader = false;
  fdgpu_engine_t *eng = nullptr;
  std::vector<uint8_t> arena;
  std::vector<fdgpu_txn_t> txns;
  std::vector<int8_t> codes;
  std::atomic<uint64_t> errors{0}, calls{0}, batches{0};
};

SyncState &sync_state() {
  /* leaked on purpose: no destructor runs at exit, after the HIP runtime may
     already be gone, or while a caller thread still waits */
  static SyncState *st = new SyncState;
  return *st;
}

constexpr uint64_t SYNC_BATCH_MAX = 4096;    /* calls per coalesced batch */
/* arena bytes of one coalesced batch: the engine's arena is opened at twice
   the batch's need (room to grow) and must stay within 32-bit offsets
   (fdgpu_engine_open), so a batch holds at most half of that; a single call
   needing more cannot run on the engine at all */
constexpr uint64_t SYNC_ARENA_LIMIT = (0xFFFFFFF0ull - FDGPU_ARENA_SLACK) / 2;
const uint64_t SYNC_ARENA_MAX = [] {
  const char *v = getenv("FDGPU_SYNC_ARENA_MAX");       /* tests: reach the piecewise path with small messages */
  const unsigned long long m = v ? strtoull(v, nullptr, 0) : 0;
  return m >= 1024 && m < SYNC_ARENA_LIMIT ? (uint64_t)m : SYNC_ARENA_LIMIT;
}();
inline uint64_t sync_need(uint64_t msg_sz, uint32_t n) { return 96ull * n + msg_sz; }

void sync_failed(SyncState &st, const char *what) {
  st.errors.fetch_add(1, std::memory_order_relaxed);
  const char *fc = getenv("FDGPU_SYNC_FAIL_CLOSED");
  if (!(fc && fc[0] == '1')) {
    fprintf(stderr, "fd_ed25519_gpu: %s: %s (FDGPU_SYNC_FAIL_CLOSED=1 rejects the calls instead)\n", what,
            fdgpu_last_error());
    abort();
  }
}

bool sync_open(SyncState &st, uint64_t need);
bool sync_run_prehashed(SyncState &st, SyncReq &r);
bool sync_fill_run(SyncState &st, const std::vector<SyncReq *> &batch, uint64_t need);

/* the leader's batch: returns false on an engine failure */
bool sync_run(SyncState &st, const std::vector<SyncReq *> &batch) {
  uint64_t need = 0;
  for (const SyncReq *r : batch) need += sync_need(r->msg_sz, r->n);
  if (need > SYNC_ARENA_MAX) {
    if (batch.size() == 1) return sync_run_prehashed(st, *batch[0]);    /* a call alone: its message in pieces */
    set_err("a batch needs %llu arena bytes (at most %llu)", (unsigned long long)need,
            (unsigned long long)SYNC_ARENA_MAX);
    return false;
  }
  if (!sync_open(st, need)) return false;
  return sync_fill_run(st, batch, need);
}

/* One call whose message exceeds a batch arena: k_i = SHA-512(R_i || A_i ||
   M) for its n signatures on the device, a piece of M (at most
   SYNC_ARENA_MAX bytes) per launch of fdgpu_sha512_stream_kernel, then the
   verify from those digests and the batch_single_msg combine -- the same
   code a batch would give it.  Buffers are the call's own (a rare path). */
bool sync_run_prehashed(SyncState &st, SyncReq &r) {
  if (!sync_open(st, 0)) return false;
  fdgpu_engine_t *e = st.eng;
  HIPCHK(hipSetDevice(e->device), false);
  const uint32_t n = r.n;
  const uint64_t sig_at = 0, pub_at = 64ull * n, st_at = (pub_at + 32ull * n + 63) & ~63ull;
  const uint64_t arena_sz = st_at + 64ull * n;
  const uint64_t piece = std::max<uint64_t>(256, SYNC_ARENA_MAX & ~127ull);
  const uint64_t per_launch = piece / 128 - 1;            /* blocks whose message bytes fit one piece */
  uint8_t *d_arena = nullptr, *d_m = nullptr, *d_ra = nullptr, *d_codes = nullptr;
  fdgpu_sig_desc_t *d_sigs = nullptr;
  fdgpu_txn_desc_t *d_txn = nullptr;
  uint32_t *d_ws = nullptr;
  bool ok = false;
  do {
    if (hipMalloc((void **)&d_arena, arena_sz + FDGPU_ARENA_SLACK) != hipSuccess ||
        hipMalloc((void **)&d_m, piece) != hipSuccess || hipMalloc((void **)&d_ra, 64ull * n) != hipSuccess ||
        hipMalloc((void **)&d_codes, 2ull * n + 32) != hipSuccess ||
        hipMalloc((void **)&d_sigs, n * sizeof(fdgpu_sig_desc_t)) != hipSuccess ||
        hipMalloc((void **)&d_txn, sizeof(fdgpu_txn_desc_t)) != hipSuccess ||
        hipMalloc((void **)&d_ws, fdgpu_ws_bytes(n)) != hipSuccess) {
      set_err("prehashed call: device allocation");
      break;
    }
    std::vector<uint8_t> h_arena(arena_sz, 0), h_ra(64ull * n);
    std::vector<fdgpu_sig_desc_t> h_sigs(n);
    for (uint32_t i = 0; i < n; i++) {
      memcpy(h_arena.data() + sig_at + 64ull * i, r.sigs + 64ull * i, 64);
      memcpy(h_arena.data() + pub_at + 32ull * i, r.pubs + 32ull * i, 32);
      memcpy(h_ra.data() + 64ull * i, r.sigs + 64ull * i, 32);        /* R */
      memcpy(h_ra.data() + 64ull * i + 32, r.pubs + 32ull * i, 32);   /* A */
      h_sigs[i] = fdgpu_sig_desc_t{(uint32_t)(st_at + 64ull * i), 0u, (uint32_t)(sig_at + 64ull * i),
                                   (uint32_t)(pub_at + 32ull * i)};
    }
    const fdgpu_txn_desc_t h_txn{0u, n};
    hipStream_t s = e->compute;
    if (hipMemcpyAsync(d_arena, h_arena.data(), arena_sz, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d_ra, h_ra.data(), 64ull * n, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d_sigs, h_sigs.data(), n * sizeof(fdgpu_sig_desc_t), hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d_txn, &h_txn, sizeof h_txn, hipMemcpyHostToDevice, s) != hipSuccess) {
      set_err("prehashed call: upload");
      break;
    }
    const uint64_t total = fdgpu_sha512_stream_blocks(r.msg_sz);
    bool hashed = true;
    for (uint64_t b0 = 0; b0 < total && hashed; b0 += per_launch) {
      const uint64_t b1 = std::min(total, b0 + per_launch);
      /* the message bytes of blocks [b0, b1): M[128 b0 - 64, 128 b1 + 64) within M */
      const uint64_t m0 = b0 ? 128 * b0 - 64 : 0, m1 = std::min<uint64_t>(r.msg_sz, 128 * b1 + 64);
      const uint64_t mlen = m1 > m0 ? m1 - m0 : 0;
      hashed = (!mlen || hipMemcpyAsync(d_m, r.msg + m0, mlen, hipMemcpyHostToDevice, s) == hipSuccess) &&
               fdgpu_launch_sha512_stream(d_m, m0, mlen, r.msg_sz, b0, (uint32_t)(b1 - b0), d_ra,
                                          (uint64_t *)(d_arena + st_at), n, s) == hipSuccess &&
               hipStreamSynchronize(s) == hipSuccess;              /* the piece buffer is reused next */
    }
    if (!hashed) { set_err("prehashed call: hashing"); break; }
    int8_t code = 0;
    if (fdgpu_launch_verify_prehashed(d_arena, d_sigs, n, e->d_btab, d_ws, (int8_t *)d_codes, kflags(e), s) !=
            hipSuccess ||
        fdgpu_launch_combine(d_txn, 1, (const int8_t *)d_codes, (int8_t *)d_codes + n + 16, nullptr, s) !=
            hipSuccess ||
        hipMemcpyAsync(&code, d_codes + n + 16, 1, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      set_err("prehashed call: verify");
      break;
    }
    r.code = code;
    ok = true;
  } while (0);
  (void)hipStreamSynchronize(e->compute);
  for (void *p : {(void *)d_arena, (void *)d_m, (void *)d_ra, (void *)d_codes, (void *)d_sigs, (void *)d_txn,
                  (void *)d_ws})
    if (p) (void)hipFree(p);
  return ok;
}

/* the coalesced batch's engine, (re)opened for a batch needing `need` arena
   bytes (0: as it is) */
bool sync_open(SyncState &st, uint64_t need) {
  if (!st.eng || need > st.eng->cfg.max_arena) {
    if (st.eng) fdgpu_engine_close(st.eng);
    fdgpu_cfg_t cfg{};
    cfg.max_txn = SYNC_BATCH_MAX; cfg.max_sig = SYNC_BATCH_MAX * 16; cfg.ring_depth = 1;
    /* a call's batch is small (one txn per concurrent caller): the two-lane
       kernel's shorter wave is the call's latency (FDGPU_SYNC_PAIR=0: off) */
    const char *sp = getenv("FDGPU_SYNC_PAIR");
    cfg.flags = (sp && sp[0] == '0') ? 0u : FDGPU_FLAG_PAIR_AUTO | FDGPU_FLAG_SPREAD_AUTO;
    cfg.max_arena = std::min<uint64_t>(std::max<uint64_t>(SYNC_BATCH_MAX * (96 * 16 + 1232), need * 2),
                                       2 * SYNC_ARENA_LIMIT);
    const char *dv = getenv("FDGPU_SYNC_DEVICE");
    st.eng = fdgpu_engine_open(dv ? atoi(dv) : 0, &cfg);
    if (!st.eng) return false;
  }
  return true;
}

/* the batch's calls into the arena, one txn each, verified on the engine */
bool sync_fill_run(SyncState &st, const std::vector<SyncReq *> &batch, uint64_t need) {
  st.arena.resize(need);
  st.txns.resize(batch.size());
  st.codes.resize(batch.size());
  uint64_t o = 0;
  for (size_t k = 0; k < batch.size(); k++) {
    const SyncReq &r = *batch[k];
    fdgpu_txn_t &t = st.txns[k];
    t.sig_off = (uint32_t)o; memcpy(st.arena.data() + o, r.sigs, 64ull * r.n); o += 64ull * r.n;
    t.pub_off = (uint32_t)o; memcpy(st.arena.data() + o, r.pubs, 32ull * r.n); o += 32ull * r.n;
    t.msg_off = (uint32_t)o; if (r.msg_sz) memcpy(st.arena.data() + o, r.msg, r.msg_sz); o += r.msg_sz;
    t.msg_sz = (uint32_t)r.msg_sz; t.sig_cnt = r.n;
  }
  const int64_t tk = fdgpu_submit(st.eng, st.arena.data(), need, st.txns.data(), batch.size());
  if (tk < 0) return false;
  if (fdgpu_poll(st.eng, tk, st.codes.data(), 1) != FDGPU_OK) return false;
  for (size_t k = 0; k < batch.size(); k++) batch[k]->code = st.codes[k];
  return true;
}

int sync_verify(const uint8_t *msg, uint64_t msg_sz, const uint8_t *sigs, const uint8_t *pubs, uint32_t n) {
  if (n == 0 || n > 16) return FD_ED25519_ERR_SIG;            /* fd_ed25519_user.c:238-241 */
  SyncState &st = sync_state();
  st.calls.fetch_add(1, std::memory_order_relaxed);
  SyncReq req{msg, sigs, pubs, msg_sz, n};
  std::unique_lock<std::mutex> lk(st.mu);
  st.pending.push_back(&req);
  while (!req.done) {
    if (st.leader) { st.cv.wait(lk); continue; }
    st.leader = true;                          /* this thread verifies everything queued so far */
    std::vector<SyncReq *> batch;
    /* as many queued calls as fit one batch's arena; a call that fits no
       arena is taken alone (its message is then hashed in pieces) */
    size_t take = 0;
    uint64_t need = 0;
    while (take < st.pending.size() && take < SYNC_BATCH_MAX) {
      const uint64_t c = sync_need(st.pending[take]->msg_sz, st.pending[take]->n);
      if (take && need + c > SYNC_ARENA_MAX) break;
      need += c;
      take++;
    }
    batch.assign(st.pending.begin(), st.pending.begin() + (long)take);
    st.pending.erase(st.pending.begin(), st.pending.begin() + (long)take);
    lk.unlock();
    int prev_dev = -1;
    if (hipGetDevice(&prev_dev) != hipSuccess) prev_dev = -1;
    const bool ok = sync_run(st, batch);
    if (prev_dev >= 0) (void)hipSetDevice(prev_dev);
    if (!ok) {
      sync_failed(st, "verify batch failed");
      for (SyncReq *r : batch) r->code = FD_ED25519_ERR_SIG;   /* fail closed */
      if (st.eng) { fdgpu_engine_close(st.eng); st.eng = nullptr; }   /* reopened by the next batch */
    }
    st.batches.fetch_add(1, std::memory_order_relaxed);
    lk.lock();
    for (SyncReq *r : batch) r->done = true;
    st.leader = false;
    st.cv.notify_all();
  }
  return req.code;
}

}  // namespace

extern "C" {

int fd_ed25519_verify(uint8_t const msg[], uint64_t msg_sz, uint8_t const sig[64], uint8_t const public_key[32],
                      fd_sha512_t *sha) {
  (void)sha;
  return sync_verify(msg, msg_sz, sig, public_key, 1);
}

int fd_ed25519_verify_batch_single_msg(uint8_t const msg[], uint64_t const msg_sz, uint8_t const signatures[64],
                                       uint8_t const pubkeys[32], fd_sha512_t *shas[1], uint8_t const batch_sz) {
  (void)shas;
  return sync_verify(msg, msg_sz, signatures, pubkeys, batch_sz);
}

int fdgpu_ed25519_verify(uint8_t const msg[], uint64_t msg_sz, uint8_t const sig[64], uint8_t const public_key[32]) {
  return sync_verify(msg, msg_sz, sig, public_key, 1);
}

int fdgpu_ed25519_verify_batch_single_msg(uint8_t const msg[], uint64_t msg_sz, uint8_t const signatures[64],
                                          uint8_t const pubkeys[32], uint8_t batch_sz) {
  return sync_verify(msg, msg_sz, signatures, pubkeys, batch_sz);
}

void fdgpu_sync_stats(uint64_t *calls, uint64_t *batches, uint64_t *errors) {
  SyncState &st = sync_state();
  if (calls) *calls = st.calls.load(std::memory_order_relaxed);
  if (batches) *batches = st.batches.load(std::memory_order_relaxed);
  if (errors) *errors = st.errors.load(std::memory_order_relaxed);
}

uint64_t fdgpu_sync_errors(void) { return sync_state().errors.load(std::memory_order_relaxed); }

char const *fd_ed25519_strerror(int err) {
  switch (err) {
    case FD_ED25519_SUCCESS: return "success";
    case FD_ED25519_ERR_SIG: return "bad signature";
    case FD_ED25519_ERR_PUBKEY: return "bad public key";
    case FD_ED25519_ERR_MSG: return "bad message";
    default: break;
  }
  return "unknown";
}

/* --------------------------------------------------------- diagnostics */

#define DALLOC(buf, T, n) do { if (hipMalloc(&(buf).p, (size_t)(n) * sizeof(T) + 64) != hipSuccess) { \
  (buf).p = nullptr; set_err("alloc"); return FDGPU_ERR_DEVICE; } } while (0)

int fdgpu_debug_fe_ops(fdgpu_engine_t *e, uint8_t const *ab, uint64_t n, uint8_t *out) {
  if (!e || !n) return FDGPU_ERR_INVAL;
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  DevBuf din, dout;
  DALLOC(din, uint32_t, n * 16);
  DALLOC(dout, uint32_t, n * 64);
  HIPCHK(hipMemcpy(din.p, ab, n * 64, hipMemcpyHostToDevice), FDGPU_ERR_DEVICE);
  HIPCHK(fdgpu_launch_test_fe((uint32_t *)din.p, (uint32_t *)dout.p, (uint32_t)n, e->compute), FDGPU_ERR_DEVICE);
  HIPCHK(hipStreamSynchronize(e->compute), FDGPU_ERR_DEVICE);
  HIPCHK(hipMemcpy(out, dout.p, n * 256, hipMemcpyDeviceToHost), FDGPU_ERR_DEVICE);
  return FDGPU_OK;
}

int fdgpu_debug_decode(fdgpu_engine_t *e, uint8_t const *enc, uint64_t n, int ref_mapping, uint8_t *out) {
  if (!e || !n) return FDGPU_ERR_INVAL;
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  DevBuf din, dout;
  DALLOC(din, uint32_t, n * 8);
  DALLOC(dout, uint32_t, n * 18);
  HIPCHK(hipMemcpy(din.p, enc, n * 32, hipMemcpyHostToDevice), FDGPU_ERR_DEVICE);
  HIPCHK(fdgpu_launch_test_decode((uint32_t *)din.p, (uint32_t *)dout.p, (uint32_t)n,
                                  ref_mapping ? FDGPU_FLAG_REF_MAP : 0u, e->compute),
         FDGPU_ERR_DEVICE);
  HIPCHK(hipStreamSynchronize(e->compute), FDGPU_ERR_DEVICE);
  HIPCHK(hipMemcpy(out, dout.p, n * 72, hipMemcpyDeviceToHost), FDGPU_ERR_DEVICE);
  return FDGPU_OK;
}

static int debug_msgs(fdgpu_engine_t *e, uint8_t const *arena, uint64_t arena_sz, fdgpu_txn_t const *txns, uint64_t n,
                      uint8_t *out, int hram) {
  if (!e || !n) return FDGPU_ERR_INVAL;
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  std::vector<fdgpu_sig_desc_t> d(n);
  for (uint64_t i = 0; i < n; i++) {
    if ((uint64_t)txns[i].msg_off + txns[i].msg_sz > arena_sz ||
        (hram && ((uint64_t)txns[i].sig_off + 64 > arena_sz || (uint64_t)txns[i].pub_off + 32 > arena_sz))) {
      set_err("descriptor out of bounds"); return FDGPU_ERR_INVAL;
    }
    d[i].msg_off = txns[i].msg_off; d[i].msg_sz = txns[i].msg_sz;
    d[i].sig_off = txns[i].sig_off; d[i].pub_off = txns[i].pub_off;
  }
  DevBuf da, dd, dout;
  DALLOC(da, uint8_t, arena_sz + FDGPU_ARENA_SLACK);
  DALLOC(dd, fdgpu_sig_desc_t, n);
  DALLOC(dout, uint32_t, n * 16);
  HIPCHK(hipMemset(da.p, 0, arena_sz + FDGPU_ARENA_SLACK), FDGPU_ERR_DEVICE);
  if (arena_sz) HIPCHK(hipMemcpy(da.p, arena, arena_sz, hipMemcpyHostToDevice), FDGPU_ERR_DEVICE);
  HIPCHK(hipMemcpy(dd.p, d.data(), n * sizeof(fdgpu_sig_desc_t), hipMemcpyHostToDevice), FDGPU_ERR_DEVICE);
  if (hram)
    HIPCHK(fdgpu_launch_test_hram((uint8_t *)da.p, (fdgpu_sig_desc_t *)dd.p, (uint32_t)n, (uint32_t *)dout.p,
                                  e->compute),
           FDGPU_ERR_DEVICE);
  else
    HIPCHK(fdgpu_launch_test_sha512((uint8_t *)da.p, (fdgpu_sig_desc_t *)dd.p, (uint32_t)n, (uint32_t *)dout.p,
                                    e->compute),
           FDGPU_ERR_DEVICE);
  HIPCHK(hipStreamSynchronize(e->compute), FDGPU_ERR_DEVICE);
  HIPCHK(hipMemcpy(out, dout.p, n * (hram ? 32 : 64), hipMemcpyDeviceToHost), FDGPU_ERR_DEVICE);
  return FDGPU_OK;
}

int fdgpu_debug_sha512(fdgpu_engine_t *e, uint8_t const *arena, uint64_t arena_sz, fdgpu_txn_t const *msgs,
                       uint64_t n, uint8_t *out) {
  return debug_msgs(e, arena, arena_sz, msgs, n, out, 0);
}

int fdgpu_debug_hram(fdgpu_engine_t *e, uint8_t const *arena, uint64_t arena_sz, fdgpu_txn_t const *txns,
                     uint64_t n, uint8_t *out) {
  return debug_msgs(e, arena, arena_sz, txns, n, out, 1);
}

int fdgpu_debug_sc_reduce(fdgpu_engine_t *e, uint8_t const *in, uint64_t n, uint8_t *out) {
  if (!e || !n) return FDGPU_ERR_INVAL;
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  DevBuf din, dout;
  DALLOC(din, uint32_t, n * 16);
  DALLOC(dout, uint32_t, n * 8);
  HIPCHK(hipMemcpy(din.p, in, n * 64, hipMemcpyHostToDevice), FDGPU_ERR_DEVICE);
  HIPCHK(fdgpu_launch_test_sc_reduce((uint32_t *)din.p, (uint32_t *)dout.p, (uint32_t)n, e->compute),
         FDGPU_ERR_DEVICE);
  HIPCHK(hipStreamSynchronize(e->compute), FDGPU_ERR_DEVICE);
  HIPCHK(hipMemcpy(out, dout.p, n * 32, hipMemcpyDeviceToHost), FDGPU_ERR_DEVICE);
  return FDGPU_OK;
}

int fdgpu_debug_hs_split(fdgpu_engine_t *e, uint8_t const *k, uint64_t n, uint8_t *out) {
  if (!e || !n) return FDGPU_ERR_INVAL;
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  DevBuf din, dout;
  DALLOC(din, uint32_t, n * 8);
  DALLOC(dout, uint32_t, n * 16);
  HIPCHK(hipMemcpy(din.p, k, n * 32, hipMemcpyHostToDevice), FDGPU_ERR_DEVICE);
  HIPCHK(fdgpu_launch_test_hs_split((uint32_t *)din.p, (uint32_t *)dout.p, (uint32_t)n, e->compute),
         FDGPU_ERR_DEVICE);
  HIPCHK(hipStreamSynchronize(e->compute), FDGPU_ERR_DEVICE);
  HIPCHK(hipMemcpy(out, dout.p, n * 64, hipMemcpyDeviceToHost), FDGPU_ERR_DEVICE);
  return FDGPU_OK;
}

int fdgpu_debug_sig_codes(fdgpu_engine_t *e, uint8_t const *arena, uint64_t arena_sz, fdgpu_txn_t const *txns,
                          uint64_t txn_cnt, int8_t *sig_codes) {
  if (!e) return FDGPU_ERR_INVAL;
  HIPCHK(hipSetDevice(e->device), FDGPU_ERR_DEVICE);
  uint64_t total = 0;
  for (uint64_t t = 0; t < txn_cnt; t++) total += (txns[t].sig_cnt >= 1 && txns[t].sig_cnt <= 16) ? txns[t].sig_cnt : 0;
  std::vector<fdgpu_sig_desc_t> sd(total + 1);
  std::vector<fdgpu_txn_desc_t> td(txn_cnt + 1);
  std::vector<uint32_t> pm(total + 1);
  uint32_t *perm = bucket(e) ? pm.data() : nullptr;
  const int64_t ns = expand(arena_sz, txns, txn_cnt, total, sd.data(), td.data(), perm);
  if (ns < 0) return FDGPU_ERR_INVAL;
  if (!ns) return FDGPU_OK;
  DevBuf da, dd, dp, dc;
  DALLOC(da, uint8_t, arena_sz + FDGPU_ARENA_SLACK);
  DALLOC(dd, fdgpu_sig_desc_t, ns);
  DALLOC(dp, uint32_t, ns);
  DALLOC(dc, int8_t, ns);
  HIPCHK(hipMemset(da.p, 0, arena_sz + FDGPU_ARENA_SLACK), FDGPU_ERR_DEVICE);
  HIPCHK(hipMemcpy(da.p, arena, arena_sz, hipMemcpyHostToDevice), FDGPU_ERR_DEVICE);
  HIPCHK(hipMemcpy(dd.p, sd.data(), ns * sizeof(fdgpu_sig_desc_t), hipMemcpyHostToDevice), FDGPU_ERR_DEVICE);
  if (perm) HIPCHK(hipMemcpy(dp.p, perm, ns * sizeof(uint32_t), hipMemcpyHostToDevice), FDGPU_ERR_DEVICE);
  const uint32_t flags = kflags(e);
  if ((uint64_t)ns > e->ws_sig) { int rc = ensure_ws(e, (uint64_t)ns); if (rc) return rc; }
  HIPCHK(fdgpu_launch_verify_sigs((uint8_t *)da.p, (fdgpu_sig_desc_t *)dd.p, (uint32_t)ns,
                                  perm ? (uint32_t *)dp.p : nullptr, e->d_btab, e->d_ws, (int8_t *)dc.p, flags,
                                  e->compute, nullptr, e->resident_blocks, e->kc_seed),
         FDGPU_ERR_DEVICE);
  HIPCHK(hipStreamSynchronize(e->compute), FDGPU_ERR_DEVICE);
  HIPCHK(hipMemcpy(sig_codes, dc.p, ns, hipMemcpyDeviceToHost), FDGPU_ERR_DEVICE);
  return FDGPU_OK;
}

}  // extern "C"
