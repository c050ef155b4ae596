/* fd_verify_tile.h -- C ABI of the verify-stage integration around the
   MI355X Ed25519 engine (libfd_verify_tile.so).

   What the reference's verify tile does per frag (src/app/fdctl/run/tiles/
   fd_verify.c:36-148, fd_verify.h:45-89): filter by round robin, copy the
   payload, fd_txn_parse it, check a tcache of recent signature tags, call
   fd_ed25519_verify_batch_single_msg, insert the tag on success, and publish
   [payload][pad to 2][fd_txn_t][u16 payload_sz] downstream with the tag as
   the frag signature.  Here the same contract is met with the signature
   work batched onto one or more GPUs:

     ingest   frags are read off a tango mcache/dcache pair with the
              reference's overrun protocol and parsed on the host into a
              batch arena;
     verify   whole batches go to the GPU engine(s) (fdgpu_submit), several
              batches in flight, round-robin over the engines of a node;
     publish  completed batches are resolved strictly in ingest order: for
              each txn the tcache is queried, a verify failure filters it,
              a success inserts the tag and publishes -- exactly the outcome
              sequence the reference's per-frag fd_txn_verify produces (the
              tcache decision only depends on earlier txns' outcomes, which
              are final by the time a txn is resolved).

   Restated wire formats (bit-compatible with the reference, so the tile can
   sit between the reference's quic and dedup tiles):
     fdt_frag_meta_t      fd_frag_meta_t          src/tango/fd_tango_base.h:146-203
     fdt_mcache_*         fd_mcache publish/wait  src/tango/mcache/fd_mcache.h:265-322,574-601
                                                  fd_mcache.c:64-69 (line init)
     fdt_dcache_*         compact chunk ring      src/tango/dcache/fd_dcache.h:198-269
     fdt_tcache_*         fd_tcache               src/tango/tcache/fd_tcache.h:34-404
     fdt_hash             fd_hash (xxhash-r39)    src/util/fd_hash.c:12-73
     fdt_txn_t/_parse     fd_txn_t, fd_txn_parse  src/ballet/txn/fd_txn.h:122-335,437-440
                                                  src/ballet/txn/fd_txn_parse.c:7-243
                                                  src/ballet/txn/fd_compact_u16.h:29-75
   Everything here is plain host C/C++; only the verify step touches the GPU
   (through libfd_ed25519_gpu.so). */
#ifndef FD_VERIFY_TILE_H
#define FD_VERIFY_TILE_H

#include <stddef.h>
#include <stdint.h>

#include "fd_ed25519_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------ constants */

#define FDT_CHUNK_LG_SZ        (6)
#define FDT_CHUNK_SZ           (64UL)
#define FDT_TPU_MTU            (1232UL)                    /* src/disco/fd_disco_base.h:34 */
#define FDT_TXN_MTU            (1232UL)                    /* src/ballet/txn/fd_txn.h:103 */
#define FDT_TXN_MAX_SZ         (852UL)                     /* fd_txn.h:98 */
#define FDT_TPU_DCACHE_MTU     (FDT_TPU_MTU + FDT_TXN_MAX_SZ + 2UL)   /* fd_disco_base.h:41 */
#define FDT_TXN_SIG_MAX        (127UL)                     /* fd_txn.h:67 */
#define FDT_TXN_ACCT_ADDR_MAX  (128UL)                     /* fd_txn.h:76 */
#define FDT_TXN_ADDR_TABLE_LOOKUP_MAX (127UL)              /* fd_txn.h:85 */
#define FDT_TXN_INSTR_MAX      (64UL)                      /* fd_txn.h:89 */
#define FDT_TXN_VLEGACY        ((uint8_t)0xFF)
#define FDT_TXN_V0             ((uint8_t)0x00)

#define FD_TXN_VERIFY_SUCCESS  ( 0)                        /* fd_verify.h:9-11 */
#define FD_TXN_VERIFY_FAILED   (-1)
#define FD_TXN_VERIFY_DEDUP    (-2)

#define FDT_VERIFY_TCACHE_DEPTH   (16UL)                   /* fd_verify.h:6-7 */
#define FDT_VERIFY_TCACHE_MAP_CNT (64UL)
#define FDT_TCACHE_TAG_NULL       (0UL)

/* ------------------------------------------------------- frag metadata */

typedef struct __attribute__((aligned(32))) {
  uint64_t seq;
  uint64_t sig;
  uint32_t chunk;
  uint16_t sz;
  uint16_t ctl;       /* som | eom<<1 | err<<2 | orig<<3 */
  uint32_t tsorig;
  uint32_t tspub;
} fdt_frag_meta_t;

uint64_t fdt_frag_meta_ctl( uint64_t orig, int som, int eom, int err );

/* mcache: `depth` (power of 2) lines; line of seq = seq & (depth-1).
   init marks every line as not-yet-published for seq0 .. seq0+depth-1. */
void     fdt_mcache_init   ( fdt_frag_meta_t * mcache, uint64_t depth, uint64_t seq0 );
void     fdt_mcache_publish( fdt_frag_meta_t * mcache, uint64_t depth, uint64_t seq, uint64_t sig,
                             uint64_t chunk, uint64_t sz, uint64_t ctl, uint64_t tsorig, uint64_t tspub );
/* One poll of FD_MCACHE_WAIT: returns 0 if seq is not yet published,
   1 with *meta filled when it is, -1 if the consumer was overrun (then
   *seq_found is a lower bound of the producer position). */
int      fdt_mcache_poll   ( fdt_frag_meta_t const * mcache, uint64_t depth, uint64_t seq,
                             fdt_frag_meta_t * meta, uint64_t * seq_found );
/* Sequence number currently in seq's line (re-check after reading a payload). */
uint64_t fdt_mcache_query  ( fdt_frag_meta_t const * mcache, uint64_t depth, uint64_t seq );

/* compact dcache addressing (chunk = 64-B units from a base address) */
uint64_t fdt_dcache_chunk_mtu ( uint64_t mtu );
uint64_t fdt_dcache_data_sz   ( uint64_t mtu, uint64_t depth );  /* bytes for depth frags of <= mtu */
uint64_t fdt_dcache_wmark     ( uint64_t chunk0, uint64_t chunk1, uint64_t mtu );
uint64_t fdt_dcache_compact_next( uint64_t chunk, uint64_t sz, uint64_t chunk0, uint64_t wmark );

/* -------------------------------------------------------------- tcache */

uint64_t fdt_tcache_map_cnt_default( uint64_t depth );
/* Footprint in bytes of a tcache (header 4 words + ring + map), same
   layout as fd_tcache_private: {magic, depth, map_cnt, oldest, ring[depth],
   map[map_cnt]}.  map_cnt 0 = default. 0 on bad parameters. */
uint64_t fdt_tcache_footprint( uint64_t depth, uint64_t map_cnt );
void *   fdt_tcache_new      ( void * mem, uint64_t depth, uint64_t map_cnt );
void     fdt_tcache_reset    ( void * tcache );
/* 1 if tag is present */
int      fdt_tcache_query    ( void const * tcache, uint64_t tag );
/* returns dup (1: already present, unchanged; 0: inserted, oldest evicted) */
int      fdt_tcache_insert   ( void * tcache, uint64_t tag );
/* fdt_tcache_insert of tags[0..n) in order; returns how many were dups
   (e.g. to bring a tcache to its steady state -- full ring, every insert
   evicting -- before a measurement) */
uint64_t fdt_tcache_insert_many( void * tcache, uint64_t const * tags, uint64_t n );
/* Cache hints for a coming insert (no effect on the contents): the map line
   a query / insert of tag starts its probe at, and the map line of the tag
   the ahead-th next insert will evict.  A deep tcache's map (4,194,302 deep:
   64 MB) misses every cache on both. */
void     fdt_tcache_prefetch      ( void const * tcache, uint64_t tag );
void     fdt_tcache_prefetch_evict( void const * tcache, uint64_t ahead );

/* A small tcache as a ring scan: the verify tile's 16-deep tcache
   (fd_verify.h:6-7) answers exactly as fdt_tcache_query / fdt_tcache_insert
   of the same depth (the map of fd_tcache.h indexes exactly the ring's
   tags; the null tag 0 always counts as present, as the map's empty slots
   match it), with one vector compare over the ring instead of probing and
   back-shifting the map.  depth 1..FDT_TAGRING_MAX. */
#define FDT_TAGRING_MAX 32
typedef struct { uint64_t tag[ FDT_TAGRING_MAX ]; uint64_t depth, oldest; } fdt_tagring_t;
void fdt_tagring_init  ( fdt_tagring_t * r, uint64_t depth );
int  fdt_tagring_query ( fdt_tagring_t const * r, uint64_t tag );   /* 1: present */
int  fdt_tagring_insert( fdt_tagring_t * r, uint64_t tag );         /* 1: was present (no change) */

/* ---------------------------------------------------------------- hash */

uint64_t fdt_hash( uint64_t seed, void const * buf, uint64_t sz );

/* ----------------------------------------------------------------- txn */

typedef struct {
  uint8_t  program_id;
  uint8_t  _padding_reserved_1;
  uint16_t acct_cnt;
  uint16_t data_sz;
  uint16_t acct_off;
  uint16_t data_off;
} fdt_txn_instr_t;

typedef struct {
  uint16_t addr_off;
  uint8_t  writable_cnt;
  uint8_t  readonly_cnt;
  uint16_t writable_off;
  uint16_t readonly_off;
} fdt_txn_acct_addr_lut_t;

typedef struct {
  uint8_t  transaction_version;
  uint8_t  signature_cnt;
  uint16_t signature_off;
  uint16_t message_off;
  uint8_t  readonly_signed_cnt;
  uint8_t  readonly_unsigned_cnt;
  uint16_t acct_addr_cnt;
  uint16_t acct_addr_off;
  uint16_t recent_blockhash_off;
  uint8_t  addr_table_lookup_cnt;
  uint8_t  addr_table_adtl_writable_cnt;
  uint8_t  addr_table_adtl_cnt;
  uint8_t  _padding_reserved_1;
  uint16_t instr_cnt;
  fdt_txn_instr_t instr[];
} fdt_txn_t;

typedef struct {
  uint64_t success_cnt;
  uint64_t failure_cnt;
  uint64_t failure_ring[ 32 ];
} fdt_txn_parse_counters_t;

uint64_t fdt_txn_footprint( uint64_t instr_cnt, uint64_t addr_table_lookup_cnt );
/* Parses payload[0,payload_sz) into out_buf (>= FDT_TXN_MAX_SZ bytes, or
   NULL to validate only).  Returns the fdt_txn_t footprint, 0 if the
   payload is not a valid transaction.  counters_opt as the reference
   (failure_ring records a reason code per failure). */
uint64_t fdt_txn_parse( uint8_t const * payload, uint64_t payload_sz, void * out_buf,
                        fdt_txn_parse_counters_t * counters_opt );

/* The footprint fdt_txn_parse would return for the payload if it parses,
   read from its counts without the structural checks (equal to the parse's
   whenever the payload is a valid transaction; 0 if the counts run past the
   payload); *sig_cnt_opt gets the leading signature count.  The verify tile
   reserves each frag's trailer with it when the GPU parses the batch. */
uint64_t fdt_txn_peek( uint8_t const * payload, uint64_t payload_sz, uint64_t * sig_cnt_opt );

/* ----------------------------------------------------------- verifiers */

/* A verifier runs fd_ed25519_verify_batch_single_msg over whole batches,
   asynchronously.  submit returns a ticket >= 0 or < 0 (FDGPU_ERR_FULL when
   no slot is free); poll returns FDGPU_OK with codes written,
   FDGPU_PENDING, or < 0. */
typedef struct {
  void *  ctx;
  int64_t (*submit)( void * ctx, uint8_t const * arena, uint64_t arena_sz, fdgpu_txn_t const * txns,
                     uint64_t txn_cnt );
  int     (*poll)  ( void * ctx, int64_t ticket, int8_t * txn_codes, int blocking );
  /* Optional zero-copy staging (NULL when unsupported): the tile copies
     frags straight into the returned (pinned) arena; a staged batch is
     polled with poll_keep and handed back with release once published. */
  uint8_t * (*stage)        ( void * ctx, uint64_t * cap );
  int64_t   (*submit_staged)( void * ctx, uint64_t arena_sz, fdgpu_txn_t const * txns, uint64_t txn_cnt );
  int       (*poll_keep)    ( void * ctx, int64_t ticket, int8_t * txn_codes, int blocking );
  int       (*release)      ( void * ctx, int64_t ticket );
  int       (*stage_cancel) ( void * ctx );
  /* Optional GPU-side parse (NULL when unsupported): batches of raw
     payloads with their trailers reserved by the caller, fdgpu_submit_frags /
     fdgpu_poll_frags semantics (include/fd_ed25519_gpu.h). */
  int64_t   (*submit_frags) ( void * ctx, uint8_t const * arena, uint64_t arena_sz, fdgpu_frag_ex_t const * frags,
                              uint64_t frag_cnt, uint64_t trailer_sz );
  int       (*poll_frags)   ( void * ctx, int64_t ticket, int8_t * codes, uint8_t * trailers, int blocking );
  /* Optional gathered frag batches (NULL when unsupported): payloads read
     where they lie, out frags written back by the verifier,
     fdgpu_submit_frags_io / fdgpu_poll_frags_io semantics. */
  int64_t   (*submit_io)    ( void * ctx, fdgpu_frag_io_t const * frags, uint64_t frag_cnt, uint8_t * out,
                              uint64_t out_sz, uint64_t hash_seed, fdgpu_link_t const * links,
                              uint64_t link_cnt );
  int       (*poll_io)      ( void * ctx, int64_t ticket, int8_t * codes, uint64_t * tags, uint16_t * out_szs,
                              int blocking );
} fdgpu_verifier_t;

/* Multi-GPU dispatcher: batches go round-robin over `engine_cnt` engines
   (one per GPU, independent queues, no collective). */
typedef struct fdgpu_dispatch fdgpu_dispatch_t;
fdgpu_dispatch_t * fdgpu_dispatch_new( fdgpu_engine_t * const * engines, uint32_t engine_cnt );
void               fdgpu_dispatch_delete( fdgpu_dispatch_t * d );
fdgpu_verifier_t   fdgpu_dispatch_verifier( fdgpu_dispatch_t * d );

/* --------------------------------------------------------- verify tile */

typedef struct {
  /* in link (quic -> verify): mcache + payload region */
  fdt_frag_meta_t const * in_mcache;
  uint64_t                in_depth;
  uint64_t                in_seq0;
  uint8_t const *         in_base;      /* address of chunk 0 */
  uint64_t                in_chunk0;    /* valid chunk range [chunk0, wmark] */
  uint64_t                in_wmark;
  /* out link (verify -> dedup) */
  fdt_frag_meta_t *       out_mcache;
  uint64_t                out_depth;
  uint64_t                out_seq0;
  uint8_t *               out_base;
  uint64_t                out_chunk0;
  uint64_t                out_wmark;
  uint64_t const *        out_fseq;     /* reliable consumer's next seq (NULL: no flow control) */
  /* tile */
  uint64_t round_robin_idx;
  uint64_t round_robin_cnt;
  uint64_t hashmap_seed;
  uint64_t tcache_depth;                /* 0: FDT_VERIFY_TCACHE_DEPTH */
  uint64_t tcache_map_cnt;              /* 0: FDT_VERIFY_TCACHE_MAP_CNT */
  uint32_t batch_txn_max;               /* txns per GPU batch */
  uint32_t inflight_max;                /* batches in flight (<= the verifier's slots) */
  uint64_t batch_wait_ns;               /* a partial batch is submitted after this long */
  uint64_t batch_sig_max;               /* signatures per batch (<= the engines' max_sig);
                                           0: 12 x batch_txn_max, the engine's default */
} fdgpu_vtile_cfg_t;

typedef struct {
  uint64_t in_frags;        /* frags seen on the in link */
  uint64_t filtered_rr;     /* not this tile's round-robin share */
  uint64_t corrupt;         /* chunk/sz out of range (reference: FD_LOG_ERR) */
  uint64_t overrun;         /* frags lost to producer overrun */
  uint64_t parse_fail;      /* fd_txn_parse rejected */
  uint64_t verify_failed;   /* FD_TXN_VERIFY_FAILED */
  uint64_t dedup;           /* FD_TXN_VERIFY_DEDUP */
  uint64_t published;       /* FD_TXN_VERIFY_SUCCESS, published downstream */
  uint64_t batches;
  uint64_t sigs;            /* signatures sent to the GPU */
  uint64_t backpressure;    /* steps that stalled on out-link credits */
  uint64_t lat_cnt;         /* batch latencies recorded (ingest of first frag -> publish) */
  uint64_t verify_errors;   /* txns of batches the verifier rejected as malformed (failed, not published) */
  /* where the tile's time goes (ingest_ns: fdgpu_vtile only) */
  uint64_t ingest_ns;       /* polling the in link, copying and parsing frags */
  uint64_t submit_ns;       /* inside the verifier's submit / stage calls (fdgpu_vmux: and the lap guard's pass before each) */
  uint64_t poll_ns;         /* inside the verifier's non-blocking polls (fdgpu_vmux: every 8th timed, x 8) */
  uint64_t no_slot_steps;   /* steps that could not open a batch: every batch or ring slot in flight */
  uint64_t polls;           /* non-blocking polls (fdgpu_vmux) */
  uint64_t poll_done_ns;    /* the part of poll_ns in polls that completed (the results' read-out) */
  uint64_t publish_ns;      /* resolving completed batches: tags, tcache, publishing (fdgpu_vmux) */
  uint64_t batch_fill_ns;   /* summed over batches: first frag taken -> submitted (fdgpu_vmux) */
  uint64_t batch_gpu_ns;    /* summed over batches: submitted -> a poll saw it complete (fdgpu_vmux) */
  uint64_t lapped;          /* gpu_parse 2: frags the producer lapped before their payload was read
                               (FDGPU_CODE_LAPPED; also counted in overrun) */
  uint64_t rescued;         /* gpu_parse 2: payloads the lap guard copied on the tile's core at submit */
  uint64_t submit_max_ns;   /* the longest single batch submit (fdgpu_vmux) */
  uint64_t stall_max_ns;    /* the longest the tile went between two of its every-64th-call polls: a
                               stalled core (descheduled, blocked in a runtime call) (fdgpu_vmux) */
  uint64_t lap_margin_min;  /* gpu_parse 2: the fewest further publishes any batch's oldest frag of a link
                               had left before the producer reuses its line, taken when the batch is seen
                               complete (so after the device's read): (oldest seq + depth - 1) - the
                               link's newest published seq, 0 if lapped; UINT64_MAX: none measured */
} fdgpu_vtile_stats_t;

typedef struct fdgpu_vtile fdgpu_vtile_t;

fdgpu_vtile_t * fdgpu_vtile_new   ( fdgpu_vtile_cfg_t const * cfg, fdgpu_verifier_t verifier );
void            fdgpu_vtile_delete( fdgpu_vtile_t * t );
/* One run-loop iteration: ingest what is available (up to one batch),
   submit due batches, resolve and publish completed ones in order.
   Returns the number of frags resolved this step, < 0 on a verifier error. */
int64_t         fdgpu_vtile_step  ( fdgpu_vtile_t * t );
/* Runs steps until `in_frags` frags have been seen on the in link and every
   batch is resolved, or timeout_s passes.  Returns 0, or < 0. */
int             fdgpu_vtile_run   ( fdgpu_vtile_t * t, uint64_t in_frags, double timeout_s );
/* Submits a partial batch and resolves everything in flight (blocking). */
int             fdgpu_vtile_flush ( fdgpu_vtile_t * t );
void            fdgpu_vtile_stats ( fdgpu_vtile_t const * t, fdgpu_vtile_stats_t * out );
/* Copies up to max recorded batch latencies (ns) into out; returns count. */
uint64_t        fdgpu_vtile_latencies( fdgpu_vtile_t const * t, uint64_t * out, uint64_t max );
/* The tile's tcache (e.g. to reset it between test phases). */
void *          fdgpu_vtile_tcache( fdgpu_vtile_t * t );
/* Per-frag outcome log (tests): for every in-link seq the tile saw, the
   FD_TXN_VERIFY_* code, or FDGPU_VTILE_LOG_* below.  Enabled by
   fdgpu_vtile_log_enable(t, max) before the first step; entries are in the
   order outcomes became final (filtered frags at ingest, verified ones at
   resolution), so sort by seq to compare with a sequential model. */
#define FDGPU_VTILE_LOG_PARSE_FAIL (1)
#define FDGPU_VTILE_LOG_FILTERED   (2)
#define FDGPU_VTILE_LOG_LOST       (3)   /* overrun or corrupt */
void            fdgpu_vtile_log_enable( fdgpu_vtile_t * t, uint64_t log_max );
uint64_t        fdgpu_vtile_log( fdgpu_vtile_t const * t, uint64_t * seqs, int8_t * codes, uint64_t max );

/* ------------------------------------------ mux (src/disco/mux/fd_mux.h) */

/* The reference's tiles are written as callbacks of its mux run loop
   (fd_mux.h:114-299, fd_mux.c:387-699); the verify tile is the vtable of
   fd_verify.c:232-246 with FD_MUX_FLAG_COPY | FD_MUX_FLAG_MANUAL_PUBLISH.
   Restated here with the same names, argument meanings and call order so a
   tile written for the reference mux runs on fdt_mux_run, and the batched
   GPU verify tile below plugs into the reference's mux unchanged. */
#define FDT_MUX_FLAG_DEFAULT        (0UL)                 /* fd_mux.h:71-73 */
#define FDT_MUX_FLAG_MANUAL_PUBLISH (1UL)
#define FDT_MUX_FLAG_COPY           (2UL)

typedef struct {                                          /* fd_mux_context_t, fd_mux.h:106-112 */
  fdt_frag_meta_t * mcache;
  uint64_t          depth;
  uint64_t *        cr_avail;
  uint64_t *        seq;
  uint64_t          cr_decrement_amount;
} fdt_mux_context_t;

typedef void (fdt_mux_during_housekeeping_fn)( void * ctx );                                   /* fd_mux.h:125 */
typedef void (fdt_mux_before_credit_fn)( void * ctx, fdt_mux_context_t * mux );                 /* :141-142 */
typedef void (fdt_mux_after_credit_fn)( void * ctx, fdt_mux_context_t * mux, int * opt_poll_in );  /* :167-169 */
typedef void (fdt_mux_before_frag_fn)( void * ctx, uint64_t in_idx, uint64_t seq, uint64_t sig,
                                       int * opt_filter );                                      /* :188-192 */
typedef void (fdt_mux_during_frag_fn)( void * ctx, uint64_t in_idx, uint64_t seq, uint64_t sig,
                                       uint64_t chunk, uint64_t sz, int * opt_filter );         /* :222-228 */
typedef void (fdt_mux_after_frag_fn)( void * ctx, uint64_t in_idx, uint64_t seq, uint64_t * opt_sig,
                                      uint64_t * opt_chunk, uint64_t * opt_sz, uint64_t * opt_tsorig,
                                      int * opt_filter, fdt_mux_context_t * mux );              /* :260-268 */
typedef void (fdt_mux_metrics_write_fn)( void * ctx );                                          /* :281 */

typedef struct {                                          /* fd_mux_callbacks_t, fd_mux.h:288-299 */
  fdt_mux_during_housekeeping_fn * during_housekeeping;
  fdt_mux_before_credit_fn *       before_credit;
  fdt_mux_after_credit_fn *        after_credit;
  fdt_mux_before_frag_fn *         before_frag;
  fdt_mux_during_frag_fn *         during_frag;
  fdt_mux_after_frag_fn *          after_frag;
  fdt_mux_metrics_write_fn *       metrics_write;
} fdt_mux_callbacks_t;

/* fd_mux_publish (fd_mux.h:484-496): publish to the mux's out mcache at
   *ctx->seq, take one credit, advance seq. */
void fdt_mux_publish( fdt_mux_context_t * ctx, uint64_t sig, uint64_t chunk, uint64_t sz, uint64_t ctl,
                      uint64_t tsorig, uint64_t tspub );

#define FDT_MUX_IN_MAX  (16UL)
#define FDT_MUX_OUT_MAX (16UL)

typedef struct {
  uint64_t                in_cnt;
  fdt_frag_meta_t const * in_mcache[ FDT_MUX_IN_MAX ];
  uint64_t                in_depth [ FDT_MUX_IN_MAX ];
  uint64_t                in_seq0  [ FDT_MUX_IN_MAX ];
  uint64_t *              in_fseq  [ FDT_MUX_IN_MAX ];   /* the mux's position, for the in's producer (may be NULL) */
  fdt_frag_meta_t *       out_mcache;                    /* NULL: no out stream */
  uint64_t                out_depth;
  uint64_t                out_seq0;
  uint64_t                out_cnt;                       /* reliable consumers of the out stream */
  uint64_t const *        out_fseq [ FDT_MUX_OUT_MAX ];
  uint64_t                flags;                         /* FDT_MUX_FLAG_* */
  uint64_t                burst;                         /* frags published per in frag (>= 1) */
  uint64_t                cr_max;                        /* 0: the reference default (fd_mux.c:326-327) */
  uint64_t                lazy_iters;                    /* loop iterations between housekeeping events (0: 16) */
  struct fdt_mux_metrics * metrics;                      /* NULL, or written at every housekeeping event (below) */
} fdt_mux_cfg_t;

typedef struct {
  uint64_t in_frags;            /* frags read (before_frag called) */
  uint64_t filtered_before;     /* before_frag filtered */
  uint64_t filtered_after;      /* during/after_frag filtered */
  uint64_t overrun_polling;     /* frags skipped: the in producer lapped the mux */
  uint64_t overrun_reading;     /* frags abandoned: overwritten while being read */
  uint64_t backpressure;        /* loop iterations without credits */
  uint64_t published;           /* automatic publishes (not MANUAL_PUBLISH) */
  uint64_t loops;
} fdt_mux_stats_t;

/* The reference's metrics of a mux tile (src/disco/metrics/metrics.xml
   groups Link (in side, per in link), Stem and Tile; accumulated as
   fd_mux.c:370-379,440-451,525-697 does), written by fdt_mux_run into
   *cfg->metrics at every housekeeping event and when it halts, for an
   observer thread or process to read: housekeeping_cnt is a seqlock
   sequence (odd while a write is under way, twice the writes once done), so
   an observer reads it, copies the struct, re-reads it and retries while it
   was odd or changed (fdt_mux_metrics_snapshot does exactly that).
   Histograms are the reference's fd_histf: 16 exponential buckets between
   a min and a max, the first for samples < min, the last for >= max, and
   the sum of all samples.  Loop durations are sampled in ticks (the time
   stamp counter, tick_per_ns below) between 50 ns and 50 us; fragment sizes
   between 0 and 2094 bytes.  Per-iteration timing costs a counter read per
   loop iteration, so it runs only when metrics is non-NULL. */
#define FDT_HISTF_BUCKET_CNT (16UL)
typedef struct {
  uint64_t counts[ FDT_HISTF_BUCKET_CNT ];
  uint64_t sum;
  uint64_t left_edge[ FDT_HISTF_BUCKET_CNT + 1 ];   /* bucket b holds left_edge[b] <= x < left_edge[b+1] */
} fdt_histf_t;
/* fd_histf_new's bucket edges for [min, max) (fd_histf.h:77-117) */
void fdt_histf_init  ( fdt_histf_t * h, uint64_t min, uint64_t max );
void fdt_histf_sample( fdt_histf_t * h, uint64_t value );

typedef struct {                                 /* metrics.xml <group name="Link" linkside="in"> */
  uint64_t published_count;                      /* frags consumed and not filtered */
  uint64_t published_size_bytes;
  uint64_t filtered_count;
  uint64_t filtered_size_bytes;
  uint64_t overrun_polling_count;
  uint64_t overrun_polling_frag_count;
  uint64_t overrun_reading_count;
} fdt_link_in_metrics_t;

typedef struct fdt_mux_metrics {
  uint64_t tile_pid, tile_tid;                   /* <group name="Tile"> */
  uint64_t stem_in_backpressure;                 /* <group name="Stem"> gauge */
  uint64_t stem_backpressure_count;
  fdt_histf_t loop_housekeeping_duration_ticks;
  fdt_histf_t loop_backpressure_duration_ticks;
  fdt_histf_t loop_caught_up_duration_ticks;
  fdt_histf_t loop_overrun_polling_duration_ticks;
  fdt_histf_t loop_overrun_reading_duration_ticks;
  fdt_histf_t loop_filter_before_fragment_duration_ticks;
  fdt_histf_t loop_filter_after_fragment_duration_ticks;
  fdt_histf_t loop_finish_duration_ticks;
  fdt_histf_t fragment_filtered_size_bytes;
  fdt_histf_t fragment_handled_size_bytes;
  fdt_link_in_metrics_t link_in[ FDT_MUX_IN_MAX ];
  double   tick_per_ns;                          /* the "seconds" converter: seconds = ticks / tick_per_ns / 1e9 */
  uint64_t housekeeping_cnt;                     /* 2 x metrics writes so far; odd while one is under way */
} fdt_mux_metrics_t;

/* A consistent copy of *src (a metrics struct another thread or process is
   writing) into *dst; 0 on success, -1 when no stable copy was seen within
   max_tries attempts. */
int fdt_mux_metrics_snapshot( fdt_mux_metrics_t const * src, fdt_mux_metrics_t * dst, uint64_t max_tries );

/* The mux run loop (fd_mux.c:387-699) with the cnc replaced by a halt word:
   housekeeping every lazy_iters iterations (out credits from the out fseqs,
   in fseqs updated, during_housekeeping / metrics_write, halt checked);
   then before_credit; backpressure while cr_avail < cr_filt + burst;
   after_credit (poll_in 0 restarts the loop); one in polled round robin:
   overrun -> resume from the producer; before_frag; metadata read;
   during_frag; overrun while reading -> abandon (re-checked after
   during_frag as well); after_frag; automatic publish unless filtered or
   MANUAL_PUBLISH.  Runs until *halt != 0.  Returns 0, or -1 on a bad cfg. */
int  fdt_mux_run( fdt_mux_cfg_t const * cfg, fdt_mux_callbacks_t const * callbacks, void * ctx,
                  uint64_t const volatile * halt, fdt_mux_stats_t * stats_out );

/* ------------------------------- the verify tile as mux callbacks (vmux) */

/* fd_tile_verify (fd_verify.c:232-246) restated for batched GPU
   verification, run by fdt_mux_run (or the reference's fd_mux_tile) with
   FDT_MUX_FLAG_COPY | FDT_MUX_FLAG_MANUAL_PUBLISH and burst 1:
     before_frag   round-robin share (fd_verify.c:36-47);
     during_frag   copy the payload into the OUT dcache at the tile's write
                   cursor (fd_verify.c:53-74);
     after_frag    fd_txn_parse in place, append the trailer (fd_verify.c:
                   76-136), then append {msg, sigs, pubkeys, sig_cnt} to the
                   open batch -- the batch's arena IS the contiguous run of
                   out-dcache chunks its frags occupy, so with that dcache
                   registered (fdgpu_host_register) the engine DMAs it with
                   no staging copy -- and advance the cursor.  With
                   gpu_parse the tile only reads the payload's counts
                   (fdt_txn_peek) to reserve the trailer, and the frag goes
                   to the batch as {payload, trailer place}: the GPU parses,
                   and the trailer is copied in at publish;
     after_credit  poll in-flight batches (every one the verifier still
                   holds: a finished batch frees its verifier slot at once,
                   whatever its place in line) and resolve completed ones
                   strictly in ingest order (tcache query -> verify code ->
                   insert -> fdt_mux_publish of the frag where it already
                   lies), while credits last (opt_poll_in = 0 when they run
                   out); submit the open batch when full / after
                   batch_wait_ns while fewer than inflight_max batches are on
                   the verifier (up to inflight_max more may wait, finished,
                   for their turn to publish); stop polling the ins
                   (opt_poll_in = 0) while the out dcache has no room for one
                   more frag.
   Out-dcache accounting: the region from the oldest frag that may still be
   read -- published within the last cr_max - cr_avail (the mux's exposed
   count) or reserved by a batch not yet resolved -- to the write cursor is
   live; a frag is copied in only if a maximal one fits before that region.
   Size the dcache for cr_max + (2 inflight_max + 1) * batch_txn_max frags of
   FDT_TPU_DCACHE_MTU (fdgpu_vmux_dcache_data_sz) or the tile stalls early. */
typedef struct {
  uint64_t        in_cnt;
  uint8_t const * in_base  [ FDT_MUX_IN_MAX ];   /* chunk 0 address of each in link */
  uint64_t        in_chunk0[ FDT_MUX_IN_MAX ];   /* valid chunk range [chunk0, wmark] */
  uint64_t        in_wmark [ FDT_MUX_IN_MAX ];
  uint8_t *       out_base;                      /* chunk 0 address of the out dcache */
  uint64_t        out_chunk0;
  uint64_t        out_wmark;
  uint64_t        cr_max;                        /* the mux's cr_max (frags the consumers may lag) */
  uint64_t        round_robin_idx;
  uint64_t        round_robin_cnt;
  uint64_t        hashmap_seed;
  uint64_t        tcache_depth;                  /* 0: FDT_VERIFY_TCACHE_DEPTH */
  uint64_t        tcache_map_cnt;                /* 0: FDT_VERIFY_TCACHE_MAP_CNT */
  uint32_t        batch_txn_max;
  uint32_t        inflight_max;                  /* 0: 2 */
  uint64_t        batch_wait_ns;
  uint64_t        batch_sig_max;                 /* 0: 12 x batch_txn_max */
  uint64_t        batch_bytes_max;               /* arena bytes per batch (<= the engines' max_arena);
                                                    0: batch_txn_max x FDT_TPU_DCACHE_MTU rounded to chunks */
  uint32_t        gpu_parse;                     /* 1: fd_txn_parse runs on the GPU (the verifier's
                                                    submit_frags / poll_frags; required then);
                                                    2: the GPU also reads the payloads where they lie
                                                    and writes the out frags (submit_io / poll_io):
                                                    the tile touches no payload byte */
  uint32_t        _pad;
  /* gpu_parse 2: the in links' mcaches.  The device re-reads each frag's
     line after reading its payload (fdgpu_submit_frags_io's overrun
     re-check, fd_mux.c:641-655 after the copy): a frag whose line the
     producer republished before the read is dropped as overrun
     (FDGPU_CODE_LAPPED, logged LOST).  Each in dcache must hold depth + 1
     maximal frags (fdt_dcache_data_sz; checked: in_wmark - in_chunk0 >=
     depth x FDT_TPU_MTU's chunks) or be a TPU reassembly slot arena, so an
     unlapped line means an intact payload.  The mcaches must be registered
     with the verifier's engines like the dcaches. */
  fdt_frag_meta_t const * in_mcache[ FDT_MUX_IN_MAX ];
  uint64_t        in_depth [ FDT_MUX_IN_MAX ];
  /* gpu_parse 2, the lap guard: keeps the device's read of every payload
     ahead of the producer (the quic -> verify link is unreliable: the
     producer never waits, fd_frankendancer.c:131-133).
       lap_span_max  the open batch closes once it spans this many seqs of
                     any in link (0: depth / 2);
       lap_margin    at submit, a frag whose line the producer will reuse
                     within lap_margin more publishes (read in the mcache:
                     the line lap_margin behind it already holds a seq of
                     the next lap) is copied by the tile into its out frag's
                     room right away, re-checked as fd_mux.c:641-655 does,
                     and handed to the device from there (counted as
                     `rescued`; one lapped already is dropped) (0: depth / 4).
     ~0UL disables either. */
  uint64_t        lap_span_max;
  uint64_t        lap_margin;
} fdgpu_vmux_cfg_t;

typedef struct fdgpu_vmux fdgpu_vmux_t;

fdgpu_vmux_t *      fdgpu_vmux_new      ( fdgpu_vmux_cfg_t const * cfg, fdgpu_verifier_t verifier );
void                fdgpu_vmux_delete   ( fdgpu_vmux_t * t );
/* The tile's vtable (ctx = the fdgpu_vmux_t *). */
fdt_mux_callbacks_t fdgpu_vmux_callbacks( void );
/* Out dcache bytes the tile wants (see above). */
uint64_t            fdgpu_vmux_dcache_data_sz( uint64_t cr_max, uint32_t batch_txn_max, uint32_t inflight_max );
void                fdgpu_vmux_stats    ( fdgpu_vmux_t const * t, fdgpu_vtile_stats_t * out );
/* 1 when no frag is held in an open or in-flight batch. */
int                 fdgpu_vmux_idle     ( fdgpu_vmux_t const * t );
/* 0, or the verifier's fatal error (the tile then stops taking frags). */
int                 fdgpu_vmux_error    ( fdgpu_vmux_t const * t );
/* Frags whose outcome is final (published, failed, dedup, filtered, parse
   failure, corrupt); safe to read from another thread while the mux runs. */
uint64_t            fdgpu_vmux_final_cnt( fdgpu_vmux_t const * t );
/* Batch latencies (first frag ingested -> its batch resolved), ns; returns count. */
uint64_t            fdgpu_vmux_latencies( fdgpu_vmux_t const * t, uint64_t * out, uint64_t max );
/* Per-frag outcome log, as fdgpu_vtile_log (codes FD_TXN_VERIFY_* and
   FDGPU_VTILE_LOG_*). */
void                fdgpu_vmux_log_enable( fdgpu_vmux_t * t, uint64_t log_max );
uint64_t            fdgpu_vmux_log      ( fdgpu_vmux_t const * t, uint64_t * seqs, int8_t * codes, uint64_t max );

/* ---------------------------------------------------------- dedup tile */

/* src/app/fdctl/run/tiles/fd_dedup.c:89-205: consumes verify outputs (the
   parsed trailer locates signature 0), tags with fd_hash(seed, sig0, 64),
   tcache-inserts, publishes non-duplicates with sig 0. */
typedef struct {
  uint32_t                in_cnt;
  fdt_frag_meta_t const * in_mcache[ 16 ];
  uint64_t                in_depth [ 16 ];
  uint64_t                in_seq0  [ 16 ];
  uint8_t const *         in_base  [ 16 ];
  uint64_t                in_chunk0[ 16 ];
  uint64_t                in_wmark [ 16 ];
  uint32_t                unparsed_in_cnt;   /* first links carry raw txns (gossip) */
  fdt_frag_meta_t *       out_mcache;
  uint64_t                out_depth;
  uint64_t                out_seq0;
  uint8_t *               out_base;
  uint64_t                out_chunk0;
  uint64_t                out_wmark;
  uint64_t                hashmap_seed;
  uint64_t                tcache_depth;     /* reference default 4194302 (default.toml:910) */
  uint64_t                tcache_map_cnt;   /* 0: default */
  /* in link i's consumer fseq (NULL: none): the tile stores its next seq of
     link i there as it consumes (fd_fseq_update, the reliable verify -> dedup
     link of fd_topo: the verify tile's mux takes its credits from it,
     fd_mux.c:548), so a dedup tile that falls behind holds its producers
     back instead of being lapped */
  uint64_t *              in_fseq[ 16 ];
} fdgpu_dtile_cfg_t;

typedef struct {
  uint64_t in_frags, dup, published, overrun, corrupt, parse_fail;
  uint64_t done_ns;   /* fdgpu_dtile_run_sandboxed: CLOCK_MONOTONIC when the run's last frag was consumed (0: none) */
} fdgpu_dtile_stats_t;

typedef struct fdgpu_dtile fdgpu_dtile_t;
fdgpu_dtile_t * fdgpu_dtile_new   ( fdgpu_dtile_cfg_t const * cfg );
void            fdgpu_dtile_delete( fdgpu_dtile_t * t );
int64_t         fdgpu_dtile_step  ( fdgpu_dtile_t * t );   /* frags consumed this step */
void            fdgpu_dtile_stats ( fdgpu_dtile_t const * t, fdgpu_dtile_stats_t * out );
/* The dedup tile's tcache (depth cfg.tcache_depth), e.g. to fill it before a
   measurement (fdt_tcache_insert_many). */
void *          fdgpu_dtile_tcache( fdgpu_dtile_t * t );
/* Moves the tcache into memory of this process's own (huge pages where the
   host offers them), contents kept: a forked child calls it before entering
   the sandbox (fdgpu_dtile_run_sandboxed does).  0, or -1 (no memory). */
int             fdgpu_dtile_rehome( fdgpu_dtile_t * t );

/* ------------------------------------ TPU reassembly (§8(f) row 2) */

/* The quic -> verify link's producer (src/disco/quic/fd_tpu.h:20-246):
   QUIC stream data is reassembled into one of depth + burst slots of
   FDT_TPU_REASM_MTU bytes and published to an mcache of `depth` lines,
   the frag's chunk pointing into the slot.  Slots are identified by index
   (the reference hands out slot pointers).  The verify tile's in-link chunk
   range is [fdt_tpu_reasm_chunk0, fdt_tpu_reasm_wmark] (fd_verify.c:186-191). */
#define FDT_TPU_REASM_CHUNK_MTU   ((FDT_TPU_MTU + FDT_CHUNK_SZ - 1) / FDT_CHUNK_SZ)   /* 20 */
#define FDT_TPU_REASM_MTU         (FDT_TPU_REASM_CHUNK_MTU * FDT_CHUNK_SZ)             /* 1280 */
#define FDT_TPU_REASM_SUCCESS     (0)
#define FDT_TPU_REASM_ERR_SZ      (1)     /* message over FDT_TXN_MTU */
#define FDT_TPU_REASM_ERR_SKIP    (2)     /* gap in the stream data */
#define FDT_TPU_REASM_ERR_STATE   (3)     /* slot not being reassembled */
#define FDT_TPU_REASM_STATE_FREE  (0)
#define FDT_TPU_REASM_STATE_BUSY  (1)
#define FDT_TPU_REASM_STATE_PUB   (2)

uint64_t fdt_tpu_reasm_footprint( uint64_t depth, uint64_t burst );   /* 0 on bad parameters */
void *   fdt_tpu_reasm_new      ( void * mem, uint64_t depth, uint64_t burst, uint64_t orig );  /* mem 64-aligned */
void     fdt_tpu_reasm_reset    ( void * reasm );
uint64_t fdt_tpu_reasm_chunk0   ( void * reasm, void const * base );
uint64_t fdt_tpu_reasm_wmark    ( void * reasm, void const * base );
/* new stream: a FREE slot, or the least recently prepared BUSY one (cancelled) */
uint32_t fdt_tpu_reasm_prepare  ( void * reasm, uint64_t tsorig );
int      fdt_tpu_reasm_append   ( void * reasm, uint32_t slot, uint8_t const * data, uint64_t data_sz,
                                  uint64_t data_off );
/* BUSY -> PUB as frag seq; the slot mcache line seq held goes back to FREE */
int      fdt_tpu_reasm_publish  ( void * reasm, uint32_t slot, fdt_frag_meta_t * mcache, void const * base,
                                  uint64_t seq, uint64_t tspub );
void     fdt_tpu_reasm_cancel   ( void * reasm, uint32_t slot );
int      fdt_tpu_reasm_slot_state( void * reasm, uint32_t slot );     /* FDT_TPU_REASM_STATE_*, -1 */

/* ------------------------------------- other callers (§8(f) row 4) */

/* Replay: fd_executor_txn_verify (src/flamenco/runtime/fd_executor.c:
   1157-1185) for every raw transaction payloads[off[i], off[i]+sz[i]) of a
   block, batched: each is parsed (fdt_txn_parse) and verified with
   fd_ed25519_verify_batch_single_msg semantics over the verifier, in
   batches of <= batch_txn_max txns / batch_bytes_max (>= FDT_TXN_MTU)
   payload bytes, two in flight.  codes[i] = the fd_ed25519 code (0 =
   verified; fd_executor_txn_verify returns -1 for any other) or
   FDGPU_REPLAY_PARSE_FAIL.  Returns 0, or < 0 on a verifier error. */
#define FDGPU_REPLAY_PARSE_FAIL (1)
int fdgpu_replay_verify( fdgpu_verifier_t v, uint8_t const * payloads, uint64_t const * off, uint32_t const * sz,
                         uint64_t n, uint64_t batch_txn_max, uint64_t batch_bytes_max, int8_t * codes );

/* Shred FEC-set roots: fd_ed25519_verify( roots+32i, 32, sigs+64i, pub )
   (src/disco/shred/fd_fec_resolver.c:438) for n sets in batches of
   <= batch_max; pub = pubkeys (shared_pubkey: one leader key) or
   pubkeys+32i.  codes[i] = the fd_ed25519 code.  Returns 0 or < 0. */
int fdgpu_fec_roots_verify( fdgpu_verifier_t v, uint8_t const * roots, uint8_t const * sigs,
                            uint8_t const * pubkeys, int shared_pubkey, uint64_t n, uint64_t batch_max,
                            int8_t * codes );

/* --------------------------------------- process separation (§8(f) row 1) */

/* A link (mcache + compact dcache + consumer fseq) formatted inside one
   caller-mapped region (e.g. a /dev/shm file), so that the engine process
   and sandboxed tiles in other processes can join it -- the role fd_wksp
   plays for the reference's tango objects.  mem must be 4096-aligned. */
typedef struct {
  fdt_frag_meta_t * mcache;
  uint64_t          depth;
  uint64_t          seq0;
  uint64_t          mtu;
  uint8_t *         base;      /* chunk 0 */
  uint64_t          chunk0;
  uint64_t          wmark;
  uint64_t *        fseq;      /* reliable consumer's next seq */
} fdt_link_t;

uint64_t fdt_link_footprint( uint64_t depth, uint64_t mtu );   /* 0 on bad parameters */
int      fdt_link_new      ( void * mem, uint64_t depth, uint64_t mtu, uint64_t seq0 );
/* The same with the dcache's data size given (0: fdt_dcache_data_sz(mtu,
   depth)): the verify mux tile's out dcache also holds its batches in
   flight (fdgpu_vmux_dcache_data_sz).  data_sz is rounded up to 64 B and
   must hold two mtu-sized frags. */
uint64_t fdt_link_footprint_sz( uint64_t depth, uint64_t mtu, uint64_t data_sz );
int      fdt_link_new_sz      ( void * mem, uint64_t depth, uint64_t mtu, uint64_t seq0, uint64_t data_sz );
int      fdt_link_join     ( void * mem, fdt_link_t * out );   /* 0, or -1 if not a formatted link */

/* Enters the tiles' seccomp policy (src/app/fdctl/run/tiles/
   verify.seccomppolicy, dedup.seccomppolicy): from here on only write to fd
   2 / logfile_fd, fsync(logfile_fd), clock_gettime and exit are allowed;
   any other syscall kills the process.  Returns 0 or -errno. */
int      fdt_sandbox_enter ( int logfile_fd );
/* The engine process's policy (fdt_sandbox.cpp): after its engines are
   open, warmed and registered, every thread of the process may only use the
   resource-neutral syscalls a running HIP runtime and the tiles need, ioctl
   only on dev_fds (the device fds it holds: /dev/kfd, /dev/dri/renderD*),
   clone only for threads; anything else (open, socket, exec, fork, ...)
   kills the process.  report != 0 (bring-up, tests): such a syscall fails
   with EPERM instead of killing, and is recorded (fdt_sandbox_report); it is
   never carried out either way.  Returns 0 or -errno. */
int      fdt_sandbox_engine_enter( int const * dev_fds, int dev_fd_cnt, int report );
/* The GPU driver's fds this process holds (/proc/self/fd entries naming
   /dev/kfd or /dev/dri/...), ascending, into out[0..max): the dev_fds of
   fdt_sandbox_engine_enter.  Returns the count, or -errno (-ENOSPC: more
   than max). */
int      fdt_sandbox_driver_fds( int * out, int max );
/* Report mode: bits8[k] bit j set = syscall 64 k + j was refused; returns
   how many calls were refused. */
uint64_t fdt_sandbox_report( uint64_t * bits8 );
/* Runs a dedup tile inside the sandbox until frag_target frags were
   consumed (or lost to overrun) or none arrived for idle_ns_max; writes the
   final stats to stats_out (shared memory) and exits the calling process
   with 0 (target reached), 1 (idle) or 3 (sandbox failed).  Never returns:
   call it in a child process. */
void     fdgpu_dtile_run_sandboxed( fdgpu_dtile_t * t, uint64_t frag_target, uint64_t idle_ns_max,
                                    fdgpu_dtile_stats_t * stats_out, int logfile_fd );

/* ------------------------------------------------------- frag producer */

/* A line-rate producer thread standing in for the quic tile: publishes
   payload i (arena + off[i], sz[i] bytes) as frag seq0+i into an mcache /
   compact dcache at `rate_tps` frags per second (0 = as fast as possible),
   without backpressure (the quic -> verify link has none, fd_tpu.h:52-68). */
typedef struct fdgpu_producer fdgpu_producer_t;
fdgpu_producer_t * fdgpu_producer_start( fdt_frag_meta_t * mcache, uint64_t depth, uint64_t seq0,
                                         uint8_t * base, uint64_t chunk0, uint64_t wmark,
                                         uint8_t const * arena, uint64_t const * off, uint32_t const * sz,
                                         uint64_t cnt, double rate_tps );
/* Waits for the producer; returns frags published, *elapsed_s the time it
   spent publishing them (first frag to last; a paced producer's counter
   calibration before the first frag is not counted). */
uint64_t           fdgpu_producer_join ( fdgpu_producer_t * p, double * elapsed_s );
/* 1 once the producer has published its last frag (join does not block then). */
int                fdgpu_producer_done ( fdgpu_producer_t const * p );

#ifdef __cplusplus
}
#endif

#endif /* FD_VERIFY_TILE_H */
