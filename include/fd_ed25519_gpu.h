/* fd_ed25519_gpu.h -- C ABI of the MI355X batched Ed25519 verify engine
   (libfd_ed25519_gpu.so).  Plain C types only; no HIP or torch types.

   Two surfaces:

   (i) Drop-in synchronous API with the reference's prototypes and codes:
         fd_ed25519_verify                  replaces src/ballet/ed25519/fd_ed25519.h:96-101
                                            (impl fd_ed25519_user.c:135-230)
         fd_ed25519_verify_batch_single_msg replaces src/ballet/ed25519/fd_ed25519.h:124-130
                                            (impl fd_ed25519_user.c:232-310)
         fd_ed25519_strerror                replaces src/ballet/ed25519/fd_ed25519.h:132-136
                                            (impl fd_ed25519_user.c:312-322)
       Served by the GPU engine (device 0, opened on first use); results
       are bit-identical to the reference's AVX-512 build.
       LATENCY: each call is one GPU round trip, ~0.5 ms (measured p50/p99
       514-517/523-529 us on MI355X, bench.py `sync_call_latency_*`: the
       two-lane verify kernel's one-wave lifetime plus launches and
       read-back; FDGPU_SYNC_PAIR=0: the one-lane kernel, 690/710 us), against
       ~33 us for the reference's CPU verify.  Concurrent callers are
       coalesced into one batch per round trip (group commit), so throughput
       grows with the number of calling threads.  Latency-bound callers
       (TLS handshakes, gossip, repair, the precompile) should keep the
       reference's CPU fd_ed25519_verify; INTEGRATION.md 1 shows how both
       link into one process (the fdgpu_ed25519_* names below).
       The caller thread's current HIP device is preserved.  Any msg_sz is
       verified, as the reference's (fd_ed25519_user.c:205-207): a message
       beyond one batch arena (32-bit offsets, ~2 GB) is hashed on the GPU in
       arena-sized pieces, then verified from its digests.  The reference
       API returns verify codes only and never rejects a good signature, so
       an engine failure (no GPU, a HIP error) aborts the process with the
       reason on stderr.
       FDGPU_SYNC_FAIL_CLOSED=1 in the environment makes every call of the
       failed batch return FD_ED25519_ERR_SIG instead (fdgpu_sync_errors()
       counts the failures).  FDGPU_SYNC_DEVICE=<n> selects the device
       (default 0).

   (ii) Asynchronous batch API for the verify stage (the north-star shim;
       SURVEY.md §8(b)(ii)).  One engine per GPU; each engine owns pinned,
       double-buffered host/device rings and HIP streams.  A batch is a flat
       payload arena plus per-transaction descriptors with
       fd_ed25519_verify_batch_single_msg semantics per transaction (the
       verify tile's fd_txn_verify call, src/app/fdctl/run/tiles/fd_verify.h:75).
       Result per transaction: exactly the code the reference would return.

   Threading: the ring API (submit / stage / poll / release / register) is
   thread-safe per engine; the synchronous API is thread-safe and coalesces
   concurrent calls. */
#ifndef FD_ED25519_GPU_H
#define FD_ED25519_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Result codes: identical values to src/ballet/ed25519/fd_ed25519.h:11-14 */
#define FD_ED25519_SUCCESS    ( 0)
#define FD_ED25519_ERR_SIG    (-1)
#define FD_ED25519_ERR_PUBKEY (-2)
#define FD_ED25519_ERR_MSG    (-3)

/* ------------------------------------------------------------------ (i) */

/* Opaque: the reference passes caller-owned SHA-512 scratch objects
   (fd_sha512_t, src/ballet/sha512/fd_sha512.h:15-31).  The GPU engine hashes
   on the device and never touches them; any pointer (or NULL) is accepted. */
typedef struct fd_sha512_private fd_sha512_t;

int fd_ed25519_verify( uint8_t const   msg[],        /* msg_sz bytes; NULL allowed iff msg_sz==0 */
                       uint64_t        msg_sz,
                       uint8_t const   sig[ 64 ],
                       uint8_t const   public_key[ 32 ],
                       fd_sha512_t *   sha );

int fd_ed25519_verify_batch_single_msg( uint8_t const   msg[],
                                        uint64_t const  msg_sz,
                                        uint8_t const   signatures[ 64 ],  /* 64*batch_sz */
                                        uint8_t const   pubkeys[ 32 ],     /* 32*batch_sz */
                                        fd_sha512_t *   shas[ 1 ],         /* batch_sz, unused */
                                        uint8_t const   batch_sz );

char const * fd_ed25519_strerror( int err );

/* The same two calls under engine-prefixed names, so a process can link the
   reference's CPU fd_ed25519_user.c for its latency-bound callers and call
   the GPU from its batch callers (no symbol clash). */
int fdgpu_ed25519_verify( uint8_t const msg[], uint64_t msg_sz, uint8_t const sig[ 64 ],
                          uint8_t const public_key[ 32 ] );
int fdgpu_ed25519_verify_batch_single_msg( uint8_t const msg[], uint64_t msg_sz, uint8_t const signatures[ 64 ],
                                           uint8_t const pubkeys[ 32 ], uint8_t batch_sz );
/* Counters of the synchronous API: calls, GPU batches they were coalesced
   into, and engine failures answered with FD_ED25519_ERR_SIG (any out
   pointer may be NULL). */
void     fdgpu_sync_stats( uint64_t * calls, uint64_t * batches, uint64_t * errors );
uint64_t fdgpu_sync_errors( void );

/* ----------------------------------------------------------------- (ii) */

/* One transaction of a batch (same layout as the oracle's test records):
   signatures and public keys are sig_cnt contiguous 64-B / 32-B records;
   the message is msg_sz bytes.  All offsets index the batch arena. */
typedef struct {
  uint32_t msg_off;
  uint32_t msg_sz;
  uint32_t sig_off;
  uint32_t pub_off;
  uint32_t sig_cnt;     /* verified iff 1 <= sig_cnt <= 16, else FD_ED25519_ERR_SIG */
} fdgpu_txn_t;

typedef struct fdgpu_engine fdgpu_engine_t;

typedef struct {
  uint64_t max_txn;       /* per batch */
  uint64_t max_sig;       /* per batch (sum of sig_cnt); 0 = 12 x max_txn (FD_TXN_ACTUAL_SIG_MAX);
                             a batch with more signatures is rejected with FDGPU_ERR_INVAL */
  uint64_t max_arena;     /* per batch, bytes */
  uint32_t ring_depth;    /* in-flight batches (pinned staging slots), >= 1; default 2 */
  uint32_t flags;         /* FDGPU_FLAG_* */
} fdgpu_cfg_t;

#define FDGPU_FLAG_REF_MAPPING 1u  /* portable-backend (ref) error mapping instead of AVX-512 */
#define FDGPU_FLAG_NO_BUCKET   2u  /* verify signatures in transaction order (default: grouped by
                                      SHA-512 block count, codes still returned in order) */
#define FDGPU_FLAG_FULL_PATH  4u  /* diagnostics: every signature takes the full-length fallback chain
                                      (fdgpu_full_kernel), so the parity tests cover that path */
#define FDGPU_FLAG_KEY_CACHE  8u  /* decode each distinct public key of a batch once (signer reuse, e.g.
                                      vote traffic): a hash dedup + one -A table per key, copied by the
                                      other signatures of that key; same codes, faster when keys repeat,
                                      ~1% slower on 1M-signature batches of distinct keys */
#define FDGPU_FLAG_PAIR      16u  /* two GPU lanes per signature (A's and R's decode and half-size chain in
                                      adjacent lanes, the sums exchanged): ~30% shorter verify for batches
                                      that leave the GPU's wave slots idle (small / latency-bound batches),
                                      ~1.4x the work per signature, so slower on batches that fill the GPU;
                                      same codes.  Ignored with FDGPU_FLAG_KEY_CACHE */
#define FDGPU_FLAG_MERGE     64u  /* gathered frag batches (fdgpu_submit_frags_io): the verifies of the batches
                                      ready at once run as ONE launch on a stream of the engine's own, each
                                      batch's gather / parse before it and its finish after it on the batch's
                                      slot stream (a verify is launched from submit and poll calls, so the
                                      caller polls; a blocking poll launches what is waiting).  Same codes */
#define FDGPU_FLAG_SPREAD    128u /* one verify block per CU (the launch reserves LDS a second block would need):
                                      concurrent small launches from several streams then spread over the CUs
                                      instead of stacking two blocks on one while others idle.  Same codes */
#define FDGPU_FLAG_SPREAD_AUTO 256u /* FDGPU_FLAG_SPREAD for a ring batch while its lanes and those of the
                                      engine's running batches fit the chip one block per CU (65,536) */
#define FDGPU_FLAG_PAIR_AUTO 32u  /* the FDGPU_FLAG_PAIR kernel for a ring batch while it and the engine's
                                      running batches hold <= 48 K signatures (launch bounds): the GPU has idle
                                      wave slots, latency is a wave's lifetime; the one-lane kernel otherwise.
                                      Same codes either way */

/* Status codes of the engine API (distinct from verify codes). */
#define FDGPU_OK            ( 0)
#define FDGPU_PENDING       ( 1)
#define FDGPU_ERR_INVAL     (-10)
#define FDGPU_ERR_DEVICE    (-11)
#define FDGPU_ERR_FULL      (-12)
#define FDGPU_ERR_TICKET    (-13)
/* a gathered batch names host memory no fdgpu_host_register call of the
   engine covers (a payload, the out range, an in link's mcache): a wiring
   error of the caller, not a malformed batch -- the verify tile stops on it */
#define FDGPU_ERR_UNREG     (-14)

/* Opens an engine on HIP device `device`.  Returns NULL on failure (no
   device, allocation failure); fdgpu_last_error() describes it. */
fdgpu_engine_t * fdgpu_engine_open( int device, fdgpu_cfg_t const * cfg );
/* Sizes every ring slot now for batches of up to n_sig signatures (0:
   max_sig) -- the verify workspace (3.2 KB per signature), the frag-batch
   and gathered-batch buffers -- instead of on the first batches that need
   them, so no batch allocates device or pinned memory inside the pipeline.
   Call with no batch in flight (FDGPU_ERR_FULL otherwise).  FDGPU_OK or < 0. */
int              fdgpu_engine_reserve( fdgpu_engine_t * e, uint64_t n_sig );
void             fdgpu_engine_close( fdgpu_engine_t * e );
char const *     fdgpu_last_error( void );

/* Stages the batch (copies arena + descriptors into the next pinned slot),
   enqueues H2D copy, the verify kernels and the D2H copy of the per-txn
   codes, and returns a ticket >= 0 without waiting for the GPU.  Blocks
   only if all ring slots are in flight.  Returns < 0 on error. */
int64_t fdgpu_submit( fdgpu_engine_t *    e,
                      uint8_t const *     arena,
                      uint64_t            arena_sz,
                      fdgpu_txn_t const * txns,
                      uint64_t            txn_cnt );

/* Polls a ticket.  FDGPU_PENDING if still running (and !blocking);
   FDGPU_OK when done, with txn_codes[0..txn_cnt) written (one verify code
   per transaction, in submission order); < 0 on error. */
int fdgpu_poll( fdgpu_engine_t * e, int64_t ticket, int8_t * txn_codes, int blocking );

/* Zero-copy staging (the verify tile's path): the caller writes the batch
   payload straight into a ring slot's pinned arena instead of handing over
   its own buffer, saving one host copy per byte.
     fdgpu_stage_acquire reserves a free slot and returns its pinned arena
       (capacity *cap bytes), or NULL when every slot is busy or one is
       already staged (one staged slot per engine);
     fdgpu_stage_submit submits the staged slot (arena_sz bytes written) with
       its descriptors -> ticket, as fdgpu_submit;
     fdgpu_poll_keep is fdgpu_poll but keeps the slot (and the payload bytes
       in its arena) reserved until fdgpu_release, so results can be
       published from the staged bytes after the codes are known. */
uint8_t * fdgpu_stage_acquire( fdgpu_engine_t * e, uint64_t * cap );
int64_t   fdgpu_stage_submit( fdgpu_engine_t * e, uint64_t arena_sz, fdgpu_txn_t const * txns, uint64_t txn_cnt );
int       fdgpu_poll_keep( fdgpu_engine_t * e, int64_t ticket, int8_t * txn_codes, int blocking );
int       fdgpu_release( fdgpu_engine_t * e, int64_t ticket );
/* Returns a staged (acquired, not submitted) slot to the ring. */
int       fdgpu_stage_cancel( fdgpu_engine_t * e );

/* Registered host memory (the mux-callback verify tile's path): the caller
   registers a long-lived region once -- e.g. the workspace holding the
   verify -> dedup dcache, into which the tile copies each frag exactly as the
   reference's during_frag does (fd_verify.c:53-74) -- and fdgpu_submit of an
   arena lying inside a registered region uploads it by DMA straight from
   there, with no staging copy.  The arena's bytes must stay unchanged until
   the batch is polled.  Regions are page-rounded and shared (reference
   counted) across the engines that register them; fdgpu_engine_close drops
   this engine's registrations.  FDGPU_OK or < 0.

   The ring API (submit, stage_*, poll*, release, host_register) is
   thread-safe per engine: several tile threads may share one engine. */
int       fdgpu_host_register  ( fdgpu_engine_t * e, void * p, uint64_t sz );
int       fdgpu_host_unregister( fdgpu_engine_t * e, void * p );

/* Device-resident path: inputs already in HBM (device pointers), codes
   written to device memory, work enqueued on `hip_stream` (a hipStream_t,
   NULL = the engine's compute stream).  d_sig_desc: per-signature
   {msg_off, msg_sz, sig_off, pub_off} (16 B each); d_txn_desc: per-txn
   {sig0, sig_cnt} (8 B each); d_arena must have 160 readable bytes of slack
   past its last payload byte.  d_sig_codes may be NULL when only the
   transaction codes are wanted (an engine-owned buffer is used). */
int fdgpu_verify_device( fdgpu_engine_t * e,
                         void const *     d_arena,
                         void const *     d_sig_desc,
                         uint64_t         sig_cnt,
                         void const *     d_txn_desc,
                         uint64_t         txn_cnt,
                         int8_t *         d_sig_codes,
                         int8_t *         d_txn_codes,
                         void *           hip_stream );

/* Device-resident batches owned by the engine: upload once (host arena +
   txn descriptors -> HBM, with the per-signature expansion done on the
   host), then verify any number of times with the inputs already in HBM.
   This is the path a GPU-side ingest (or a benchmark) uses; codes stay in
   HBM until fdgpu_dev_batch_codes copies them out. */
typedef struct fdgpu_dev_batch fdgpu_dev_batch_t;

fdgpu_dev_batch_t * fdgpu_dev_batch_upload( fdgpu_engine_t * e, uint8_t const * arena, uint64_t arena_sz,
                                            fdgpu_txn_t const * txns, uint64_t txn_cnt );
/* enqueue one verify of the batch on its queue (async): the engine's compute
   stream, or the batch's own stream after fdgpu_dev_batch_own_queue */
int  fdgpu_dev_batch_verify( fdgpu_engine_t * e, fdgpu_dev_batch_t * b );
/* gives the batch a private HIP stream and workspace (fdgpu_ws_bytes of its
   signature count), so verifies of different batches overlap on the GPU the
   way the ring slots of fdgpu_submit do; idempotent */
int  fdgpu_dev_batch_own_queue( fdgpu_engine_t * e, fdgpu_dev_batch_t * b );
/* wait for the batch's queue and copy the per-txn (and optionally per-signature) codes out */
int  fdgpu_dev_batch_codes( fdgpu_engine_t * e, fdgpu_dev_batch_t * b, int8_t * txn_codes, int8_t * sig_codes );
void fdgpu_dev_batch_free( fdgpu_engine_t * e, fdgpu_dev_batch_t * b );
/* The batch's device buffers, in the layout fdgpu_verify_device takes (any
   out pointer may be NULL).  *d_perm is NULL unless the engine groups
   signatures by SHA-512 block count (the default): then descriptor i's code
   belongs at signature perm[i], and only the engine's own verify
   (fdgpu_dev_batch_verify) applies it -- pass such descriptors to
   fdgpu_verify_device only from an engine opened with FDGPU_FLAG_NO_BUCKET. */
int  fdgpu_dev_batch_device_ptrs( fdgpu_dev_batch_t const * b, void ** d_arena, void ** d_sig_desc,
                                  void ** d_perm, void ** d_txn_desc, int8_t ** d_sig_codes,
                                  int8_t ** d_txn_codes );
/* signatures of the batch; for a frag batch (below) the count its last
   verify produced on the device (waits for that verify; 0 before one) */
uint64_t fdgpu_dev_batch_sig_cnt( fdgpu_dev_batch_t const * b );
/* Times `iters` back-to-back verifies of the batch on the compute stream
   with HIP events: *wall_ms = first-to-last event span (all launches),
   *verify_kernel_ms = mean duration of the signature kernel alone,
   *combine_kernel_ms = mean duration of the per-txn combine kernel. */
int  fdgpu_dev_batch_time( fdgpu_engine_t * e, fdgpu_dev_batch_t * b, int iters, double * wall_ms,
                           double * verify_kernel_ms, double * combine_kernel_ms );

/* GPU-side ingest (fd_txn_parse on the device).  A
   frag batch holds raw transaction payloads -- frag i is arena bytes
   [off, off + sz), as the verify tile receives them from the quic tile --
   and each fdgpu_dev_batch_verify runs, on the batch's queue:
   fd_txn_parse of every payload (the host parser's own source, fdt_parse.h),
   an exclusive scan of the signature counts, the per-signature expansion,
   the verify kernels and the batch_single_msg combine.  Nothing is parsed
   or expanded on the host.  A payload that is not a transaction gets
   FDGPU_CODE_PARSE_FAIL instead of a verify code. */
typedef struct {
  uint32_t off;
  uint32_t sz;          /* <= FD_TXN_MTU (1232) to parse */
} fdgpu_frag_t;
#define FDGPU_CODE_PARSE_FAIL (-64)
fdgpu_dev_batch_t * fdgpu_dev_batch_upload_frags( fdgpu_engine_t * e, uint8_t const * arena, uint64_t arena_sz,
                                                  fdgpu_frag_t const * frags, uint64_t frag_cnt );
/* Ring-slot frag batches: the verify tile's path with fd_txn_parse on the
   GPU.  Like fdgpu_submit, but the arena holds raw payloads (frag i is
   arena[off, off + sz), e.g. frags copied into a registered out dcache) and
   every txn is parsed, expanded and verified on the device.  Each frag names
   where its parsed fd_txn_t goes in a caller-sized trailer buffer:
   [tr_off, tr_off + tr_cap), tr_off 4-byte aligned, tr_cap the footprint the
   caller reserved (fdt_txn_peek in libfd_verify_tile.so reads it from the
   payload's counts without validating).  fdgpu_poll_frags returns, per frag,
   the batch_single_msg code, FDGPU_CODE_PARSE_FAIL (not a transaction), or
   FDGPU_CODE_TRAILER_CAP (parsed, but to a footprint other than tr_cap: a
   caller bug, no verdict), and copies the trailer buffer out (trailer_sz
   bytes; bytes of frags that did not parse are unspecified). */
typedef struct {
  uint32_t off;
  uint32_t sz;          /* <= FD_TXN_MTU (1232) to parse */
  uint32_t tr_off;      /* its fd_txn_t at trailers[tr_off, tr_off + tr_cap) */
  uint32_t tr_cap;
} fdgpu_frag_ex_t;
#define FDGPU_CODE_TRAILER_CAP (-65)
int64_t fdgpu_submit_frags( fdgpu_engine_t * e, uint8_t const * arena, uint64_t arena_sz,
                            fdgpu_frag_ex_t const * frags, uint64_t frag_cnt, uint64_t trailer_sz );
int     fdgpu_poll_frags  ( fdgpu_engine_t * e, int64_t ticket, int8_t * codes, uint8_t * trailers, int blocking );

/* Gathered frag batches: the verify tile's path with no payload byte touched
   on the host.  Frag i's payload lies at host address src (16-byte aligned,
   inside a region registered with fdgpu_host_register -- the quic -> verify
   dcache, where the producer wrote it) and its out frag goes to
   out[out_off, out_off + out_cap) (out inside a registered region -- the
   verify -> dedup dcache).  On the slot's stream the device reads each
   payload from host memory, parses it (fd_txn_parse), verifies it
   (batch_single_msg), tags its first signature (fd_hash(hash_seed, sig, 64),
   the dedup tag fd_verify.c publishes as the frag's sig) and writes the out
   frag exactly as the reference's after_frag lays it out in the out dcache
   (fd_verify.c:93-136): [payload][pad to 2][fd_txn_t][u16 payload_sz].
   out_cap must hold
   align2(sz) + footprint + 2; fdgpu_frag_out_cap(sz) always does (a bound
   from the size alone).  fdgpu_poll_frags_io returns per frag the code (as
   fdgpu_poll_frags: FDGPU_CODE_PARSE_FAIL, FDGPU_CODE_TRAILER_CAP when the
   parsed out frag does not fit out_cap, FDGPU_CODE_LAPPED below), the tag
   (0 unless parsed) and the out frag's size (0 unless parsed).  The finish
   kernel writes the out frags into `out` and the per-frag results into the
   slot's pinned memory in place, over the bus (no copy is queued); both are
   visible to the host once fdgpu_poll_frags_io has returned FDGPU_OK for the
   ticket, and not before.

   Overrun re-check on the device (the reference's seq re-check after its
   copy, fd_mux.c:641-655): a frag with link = i + 1 names links[i], an in
   link's mcache, and seq, the frag's sequence number on it.  After the
   device has read the payload it re-reads that mcache line's seq over the
   bus; if the producer has republished the line since (any other seq), the
   payload may be torn and the frag gets FDGPU_CODE_LAPPED (no parse, no
   verdict, no out frag).  Sound when the producer rewrites a payload only
   after the line that published it: a compact dcache of depth + 1 frags
   (fd_dcache_req_data_sz with burst 1), or the TPU reassembly slot arena
   (fd_tpu.h: a slot is freed when its line is reused).  link = 0: no
   re-check -- the caller guarantees the bytes stay unchanged until the poll
   (e.g. it copied them itself).  links / link_cnt may be NULL / 0 when no
   frag names one; each links[i].mcache must lie in a registered region. */
typedef struct {
  uint64_t src;         /* host address of the payload */
  uint32_t sz;          /* <= FD_TXN_MTU (1232) */
  uint32_t out_off;
  uint32_t out_cap;
  uint32_t link;        /* 0: no re-check; i + 1: re-check links[i]'s line of seq after the read */
  uint64_t seq;         /* the frag's seq on that link */
} fdgpu_frag_io_t;
typedef struct {
  uint64_t mcache;      /* host address of line 0 of an in link's mcache (fd_frag_meta_t, 32 B, seq first) */
  uint64_t depth;       /* its depth, a power of 2 */
} fdgpu_link_t;
#define FDGPU_LINK_MAX    (16UL)
#define FDGPU_CODE_LAPPED (-66)
uint32_t fdgpu_frag_out_cap   ( uint32_t sz );
int64_t  fdgpu_submit_frags_io( fdgpu_engine_t * e, fdgpu_frag_io_t const * frags, uint64_t frag_cnt,
                                uint8_t * out, uint64_t out_sz, uint64_t hash_seed,
                                fdgpu_link_t const * links, uint64_t link_cnt );
int      fdgpu_poll_frags_io  ( fdgpu_engine_t * e, int64_t ticket, int8_t * codes, uint64_t * tags,
                                uint16_t * out_szs, int blocking );

/* After a verify of a frag batch: frag i's parsed fd_txn_t (byte-identical to
   fd_txn_parse's output) at txn_out + i * 852 (FD_TXN_MAX_SZ; NULL: skip),
   its footprint (0: not a transaction) in txn_sz[i] (NULL: skip). */
int  fdgpu_dev_batch_txns( fdgpu_engine_t * e, fdgpu_dev_batch_t * b, void * txn_out, uint16_t * txn_sz );
/* fdgpu_dev_batch_time with the ingest kernels (parse + scan + expand of a
   frag batch; 0 for a descriptor batch) timed apart: *ingest_ms. */
int  fdgpu_dev_batch_time2( fdgpu_engine_t * e, fdgpu_dev_batch_t * b, int iters, double * wall_ms,
                            double * ingest_ms, double * verify_kernel_ms, double * combine_kernel_ms );

/* Blocks until all work enqueued on the engine's streams has finished. */
int  fdgpu_sync( fdgpu_engine_t * e );

/* Engine facts for reporting: resident workgroups (occupancy x CUs),
   threads per workgroup, workspace bytes. */
int fdgpu_engine_info( fdgpu_engine_t * e, uint32_t * grid_blocks, uint32_t * block_threads,
                       uint64_t * ws_bytes );
/* The kernels one verify launches, as a static string, e.g.
   "halfsize: fdgpu_verify_hs_kernel + fdgpu_full_kernel" (the build's path). */
char const * fdgpu_kernel_path( void );
/* The library's build, as a JSON object: every compile-time switch of the
   kernels and the engine (A/B builds change them), the fault-injection
   environment variables the engine honours, and "product": 1 iff all of them
   are at the shipped defaults.  No HIP call.  __graft_entry__.smoke() and
   bench.py refuse a library that reports "product": 0. */
char const * fdgpu_build_info( void );
/* HIP devices visible to this process (hipGetDeviceCount; starts the HIP
   runtime), or -1 when the runtime reports none / fails. */
int          fdgpu_device_count( void );

/* --------------------------------------------------------- diagnostics */

/* Where the host time of the process's last fdgpu_submit calls went (up to
   8192, oldest first): per call {staging copy, descriptor expansion, the
   rest (copies and launches enqueued)} in ns -> out[3 i .. 3 i + 2].
   Returns the number of calls written. */
uint64_t fdgpu_debug_submit_times( uint64_t * out, uint64_t max );
/* Host -> device copy rate (GB/s) of sz bytes at src (pinned or inside a
   registered region: a DMA; pageable: the runtime's staged copy) into a free
   ring slot's arena, iters copies timed with HIP events on the slot's
   stream: the PCIe ceiling beside a host-fed verify rate.  < 0 on error. */
double   fdgpu_debug_h2d_gbps( fdgpu_engine_t * e, void const * src, uint64_t sz, int iters );
/* Used by the parity tests to check each stage of the path on the GPU in
   isolation.  Host pointers; synchronous.  Return FDGPU_OK or < 0. */

/* n records of (a, b) as 2 x 32 LE bytes -> n x 8 x 32 bytes: canonical
   a*b, a^2, a+b, a-b, a^((p-5)/8), 1/a, a mod p, -a (bit 255 of inputs dropped). */
int fdgpu_debug_fe_ops( fdgpu_engine_t * e, uint8_t const * ab, uint64_t n, uint8_t * out );
/* n 32-B encodings -> n x 72 B: int32 rc (0 / -1), int32 small_order (0/1, -1 if rc),
   x (32 B canonical), y (32 B canonical). */
int fdgpu_debug_decode( fdgpu_engine_t * e, uint8_t const * enc, uint64_t n, int ref_mapping, uint8_t * out );
/* SHA-512 of n messages (arena + per-message {off, sz} as fdgpu_txn_t.msg_off/msg_sz) -> n x 64 B */
int fdgpu_debug_sha512( fdgpu_engine_t * e, uint8_t const * arena, uint64_t arena_sz,
                        fdgpu_txn_t const * msgs, uint64_t n, uint8_t * out );
/* k = SHA-512(R || A || M) mod L for n single-signature txns -> n x 32 B */
int fdgpu_debug_hram( fdgpu_engine_t * e, uint8_t const * arena, uint64_t arena_sz,
                      fdgpu_txn_t const * txns, uint64_t n, uint8_t * out );
/* n 64-B little-endian integers -> n x 32 B (x mod L) */
int fdgpu_debug_sc_reduce( fdgpu_engine_t * e, uint8_t const * in, uint64_t n, uint8_t * out );
/* the half-size scalar split of n scalars k < L (32-B little-endian each)
   on the device -> n x 64 B: |u| (20 B), |v| (20 B), then u32 ok, u_neg,
   v_neg, bits and 8 zero bytes (fdgpu_lattice.h hs_split) */
int fdgpu_debug_hs_split( fdgpu_engine_t * e, uint8_t const * k, uint64_t n, uint8_t * out );
/* per-signature codes of a batch (single-signature verify code of each
   signature, in txn order) -> sig_codes[sum sig_cnt] */
int fdgpu_debug_sig_codes( fdgpu_engine_t * e, uint8_t const * arena, uint64_t arena_sz,
                           fdgpu_txn_t const * txns, uint64_t txn_cnt, int8_t * sig_codes );

#ifdef __cplusplus
}
#endif

#endif /* FD_ED25519_GPU_H */
