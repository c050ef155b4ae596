/* fdgpu_internal.h -- declarations shared by the kernels (fdgpu_kernels.hip)
   and the host engine (fdgpu_engine.cpp).  Not part of the public C ABI. */
#pragma once

#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/fd_ed25519_gpu.h"

/* Per-signature work item (16 B, one dwordx4 per lane).  Offsets index the
   batch arena; the arena carries FDGPU_ARENA_SLACK readable bytes after
   the last payload byte. */
typedef struct {
  uint32_t msg_off;
  uint32_t msg_sz;
  uint32_t sig_off;   /* 64-B signature R || S */
  uint32_t pub_off;   /* 32-B public key */
} fdgpu_sig_desc_t;

/* Per-transaction combine item: signatures sig0 .. sig0+sig_cnt-1 of the
   signature array (batch_single_msg order).  sig_cnt outside [1,16] means
   the batch is rejected without verification (fd_ed25519_user.c:238-241). */
typedef struct {
  uint32_t sig0;
  uint32_t sig_cnt;
} fdgpu_txn_desc_t;

#define FDGPU_ARENA_SLACK   160u          /* readable bytes past the arena (SHA block loads) */
/* k in signed radix 16: 64 windows over the per-lane table {O, -A, .., -8A} */
#define FDGPU_ATAB_ENTRIES  9u            /* 0 (identity), 1A .. 8A (A negated) */
#ifndef FDGPU_ATAB_WORDS
#define FDGPU_ATAB_WORDS    40u           /* u32 per cached entry (a diagnostic build may pad it) */
#endif
/* Fixed-base comb for [S]B: S in signed radix 2^W, digit i looked up in
   table i = {0, 1, .., 2^(W-1)} x 2^(W i) B (affine niels, one 128-B line per
   entry), so [S]B costs NDIG mixed additions and no doublings.  Tables live
   in HBM (W=16: 16 x 32769 x 128 B = 67 MB, resident in the 256 MB Infinity
   Cache). */
#define FDGPU_BCOMB_BITS    16u           /* comb radix: NDIG tables of 2^(W-1)+1 entries */
#define FDGPU_BCOMB_NDIG    ((254u + FDGPU_BCOMB_BITS - 1u) / FDGPU_BCOMB_BITS)   /* covers S < 2^253 + carry */
#define FDGPU_BCOMB_ENTRIES ((1u << (FDGPU_BCOMB_BITS - 1u)) + 1u)
#define FDGPU_BCOMB_STRIDE  32u           /* u32 per entry (30 used): one 128-B line */
#define FDGPU_BCOMB_CHUNK   64u           /* entries per lane in the table build (one batch inversion) */
/* The verify equation with half-size scalars (fdgpu_lattice.h).  Per-lane
   workspace entries (cached form, 40 words each): */
#define HS_MAX_WIN          40u           /* radix-16 windows of |u|, |v| (< 2^159) */
/* A table's identity entry (digit 0) is one shared constant (g_tab_ident),
   so a lane stores entries 1..8 of each table */
#define FDGPU_TAB_STORED    (FDGPU_ATAB_ENTRIES - 1u)
                                          /* entries 0..7: 1..8 of the -A table */
#define FDGPU_WS_RTAB       FDGPU_TAB_STORED            /* entries 8..15: 1..8 of the -R table */
#define FDGPU_WS_PARK       (2u * FDGPU_TAB_STORED)     /* entry: k digits, decoded R, code (full path) */
#define FDGPU_WS_SB         (FDGPU_WS_PARK + 1u)        /* entry: [w]B (or [S]B) in cached form */
#define FDGPU_WS_ENTRIES    (FDGPU_WS_SB + 1u)          /* 18 entries: 2880 B per signature */
#define FDGPU_WS_LANE_WORDS (FDGPU_WS_ENTRIES * FDGPU_ATAB_WORDS)
#define FDGPU_BLOCK         256u
#define FDGPU_FLAG_REF_MAP  1u            /* portable-backend error mapping */
#define FDGPU_FLAG_KFULL    2u            /* half-size path: every lane takes the full-length fallback */
#define FDGPU_FLAG_KCACHE   4u            /* half-size path: one -A decode + table per distinct key */
#define FDGPU_FLAG_KPAIR    8u            /* half-size path, two lanes per signature (fdgpu_verify_pair_kernel) */
#define FDGPU_FLAG_KSPREAD  16u           /* one verify block per CU: dynamic LDS that leaves no room for a second */
/* the verify block's static LDS is 80 KB (two fill a CU's 160 KB), the
   two-lane block's 40 KB: these make one block per CU the most that fits */
#define FDGPU_SPREAD_LDS       1024u
#define FDGPU_SPREAD_LDS_PAIR  (40u * 1024u + 1024u)
/* The verify blocks (two 256-VGPR waves per SIMD) fill every SIMD's register
   file, so a kernel queued behind or beside a running verify starts its
   workgroups only as verify blocks retire: a launch of many workgroups then
   waits through many retirements before its last one runs (rocprofv3, host-fed
   1M batches: an empty fallback launch of 512 blocks took 0.8 ms, the 3,907-
   block combine 0.66 ms; profiles/r05/hostfed_trace.md).  The short kernels
   around the verify therefore run on few, fat workgroups that stride over
   their work: */
#define FDGPU_FULL_BLOCKS   16u           /* the fallback chain: its queue is ~empty (split failures ~2^-30) */
#define FDGPU_AUX_BLOCKS    64u           /* combine */
/* The gathered batches' ingest and finish: a workgroup resident beside the
   verify holds a verify block's slot on its CU for its whole life (its waves
   take VGPRs the second verify wave needs), and these kernels wait on the bus,
   so their slot time -- not their own duration -- is what the verify loses.
   16 blocks that each keep more bus accesses in flight cost a quarter of the
   slot time of 64 and still fill PCIe (profiles/r05/ubench_pcie.jsonl: 16 x
   256 threads read 57 GB/s): engine-only gathered capacity, two engines,
   69 -> 81 M txn/s, and two cfg1 tiles 58.8 -> 71.5 M
   (profiles/r05/aux_blocks.md).  FDGPU_AUX_BLOCKS_IN / _FIN override. */
#define FDGPU_IO_BLOCKS     16u
/* SHA-512 block-count groups of the host-side bucketing (expand): messages of
   more blocks than this share the last group */
#define FDGPU_NBLK_GROUPS   32u

#ifdef __cplusplus
extern "C" {
#endif

/* launchers (fdgpu_kernels.hip); all asynchronous on `stream` unless noted */
size_t     fdgpu_btab_bytes(void);                                   /* fixed-base table size */
/* builds the fixed-base table into d_btab (fdgpu_btab_bytes()); synchronous */
hipError_t fdgpu_btab_build(uint32_t *d_btab, hipStream_t stream);
/* one signature per lane; d_ws must hold fdgpu_ws_bytes(n_sig) bytes */
/* d_perm (NULL = identity): d_sig_codes[d_perm[i]] receives the code of
   descriptor i (descriptors grouped by SHA-512 block count, codes in the
   caller's order) */
/* d_n_sig != NULL: the signature count is read on the device (it is produced
   there by the GPU-side ingest); n_sig is then an upper bound that sizes the
   grid (and the workspace).  resident_blocks: verify-kernel blocks the
   device keeps resident (occupancy x CUs, the fallback kernel's grid cap);
   kc_seed: the key cache's hash seed (FDGPU_FLAG_KCACHE). */
hipError_t fdgpu_launch_verify_sigs(const uint8_t *d_arena, const fdgpu_sig_desc_t *d_sigs, uint32_t n_sig,
                                    const uint32_t *d_perm, const uint32_t *d_btab, uint32_t *d_ws,
                                    int8_t *d_sig_codes, uint32_t flags, hipStream_t stream,
                                    const uint32_t *d_n_sig, uint32_t resident_blocks, uint64_t kc_seed,
                                    int cnt_zeroed = 0);
/* The synchronous API's messages too large for one arena: SHA-512(R_i ||
   A_i || M) of n <= 64 signatures over one message, a piece of M per launch
   (blocks [blk0, blk0 + nblk) of fdgpu_sha512_stream_blocks(msg_sz); d_mbuf
   = M[m0, m0 + mlen) covering those blocks' message bytes; d_ra = n x (R ||
   A); d_state = n x 8 words), then the verify from those states
   (descriptor i: msg_off = the offset of state i in d_arena, 8-B aligned). */
uint64_t   fdgpu_sha512_stream_blocks(uint64_t msg_sz);
hipError_t fdgpu_launch_sha512_stream(const uint8_t *d_mbuf, uint64_t m0, uint64_t mlen, uint64_t msg_sz,
                                      uint64_t blk0, uint32_t nblk, const uint8_t *d_ra, uint64_t *d_state,
                                      uint32_t n, hipStream_t stream);
hipError_t fdgpu_launch_verify_prehashed(const uint8_t *d_arena, const fdgpu_sig_desc_t *d_sigs, uint32_t n_sig,
                                         const uint32_t *d_btab, uint32_t *d_ws, int8_t *d_sig_codes, uint32_t flags,
                                         hipStream_t stream);
/* the verify launch's queue counter for an n_sig grid in d_ws: a caller whose
   earlier kernel on the stream zeroes it passes cnt_zeroed (no memset) */
uint32_t  *fdgpu_verify_cnt_word(uint32_t *d_ws, uint32_t n_sig);
/* One batch of a merged verify launch (FDGPU_FLAG_MERGE): what
   fdgpu_launch_verify_sigs takes per batch, read by each block from a table
   in pinned host memory (blockIdx.y picks the batch). */
typedef struct {
  const uint8_t *arena;
  const fdgpu_sig_desc_t *sigs;
  const uint32_t *n_sig;       /* the count, produced on the device (parse + expand) */
  uint32_t *ws;                /* the batch's workspace; its fallback queue and counter follow the lanes */
  int8_t *codes;
  uint32_t *queue, *cnt;
  uint32_t bound;              /* the launch bound of the count: the batch's blocks */
  uint32_t slow;               /* fallback blocks */
} fdgpu_mbatch_t;
/* one verify (one lane per signature) + one fallback launch over nb batches:
   grids {max blocks, nb} */
hipError_t fdgpu_launch_verify_multi(const fdgpu_mbatch_t *mb, uint32_t nb, uint32_t grid_max, uint32_t slow_max,
                                     const uint32_t *d_btab, uint32_t flags, hipStream_t stream);
/* d_accept (NULL: not written): ceil(n_txn / 64) words, bit t = txn t verified */
hipError_t fdgpu_launch_combine(const fdgpu_txn_desc_t *d_txns, uint32_t n_txn, const int8_t *d_sig_codes,
                                int8_t *d_txn_codes, uint64_t *d_accept, hipStream_t stream);
hipError_t fdgpu_verify_occupancy(int *blocks_per_cu);
/* the kernels' compile-time switches as JSON members into buf; 1 iff all are
   at the shipped defaults */
int        fdgpu_kernel_build_info(char *buf, size_t n);
size_t     fdgpu_ws_bytes(uint64_t n_sig);

/* test/diagnostic kernels */
hipError_t fdgpu_launch_test_fe(const uint32_t *d_in, uint32_t *d_out, uint32_t n, hipStream_t stream);
hipError_t fdgpu_launch_test_decode(const uint32_t *d_enc, uint32_t *d_out, uint32_t n, uint32_t flags, hipStream_t stream);
hipError_t fdgpu_launch_test_sha512(const uint8_t *d_arena, const fdgpu_sig_desc_t *d_msgs, uint32_t n,
                                    uint32_t *d_out, hipStream_t stream);
hipError_t fdgpu_launch_test_hram(const uint8_t *d_arena, const fdgpu_sig_desc_t *d_sigs, uint32_t n,
                                  uint32_t *d_out, hipStream_t stream);
hipError_t fdgpu_launch_test_sc_reduce(const uint32_t *d_in, uint32_t *d_out, uint32_t n, hipStream_t stream);
/* GPU-side ingest: parse n raw payloads (frags index d_arena), scan the
   signature counts, expand the descriptors; the batch's signature count is
   left in *d_n_sig.  Buffers: d_txn_out n x FDT_TXN_MAX_SZ, d_txn_sz /
   d_txd / d_cnt / d_sig0 / d_tds n entries, d_blocktot ceil(n / 1024),
   d_sigs the sum of fdgpu_frag_sig_bound over the frags. */
uint64_t   fdgpu_frag_sig_bound(uint32_t sz);
/* d_frags: n records of frag_stride u32 words whose first two are {off, sz}
   (fdgpu_frag_t: 2, fdgpu_frag_ex_t: 4) */
hipError_t fdgpu_launch_frag_ingest(const uint8_t *d_arena, const void *d_frags, uint32_t frag_stride, uint32_t n,
                                    uint8_t *d_txn_out, uint16_t *d_txn_sz, fdgpu_txn_t *d_txd, uint32_t *d_cnt,
                                    uint32_t *d_sig0, uint32_t *d_blocktot, uint32_t *d_n_sig,
                                    fdgpu_sig_desc_t *d_sigs, fdgpu_txn_desc_t *d_tds, hipStream_t stream);
hipError_t fdgpu_launch_frag_codes(const uint16_t *d_txn_sz, uint32_t n, int8_t *d_codes, hipStream_t stream);
/* fdgpu_submit_frags, in two launches for batches up to FDGPU_SMALL_SCAN_MAX
   txns (parse, then scan + expand in one block; larger batches take
   fdgpu_launch_frag_ingest's path), and the batch's end in one launch
   (combine + parse failures + trailer pack; codes at d_codes, trailers at
   d_trailers). */
#define FDGPU_SMALL_SCAN_MAX 65536u
hipError_t fdgpu_launch_frag_ring(const uint8_t *d_arena, const fdgpu_frag_ex_t *d_fx, uint32_t n, uint8_t *d_txn_out,
                                  uint16_t *d_txn_sz, fdgpu_txn_t *d_txd, uint32_t *d_cnt, uint32_t *d_sig0,
                                  uint32_t *d_blocktot, uint32_t *d_n_sig, fdgpu_sig_desc_t *d_sigs,
                                  fdgpu_txn_desc_t *d_tds, hipStream_t stream);
hipError_t fdgpu_launch_frag_finish(const fdgpu_txn_desc_t *d_tds, uint32_t n, const int8_t *d_sig_codes,
                                    const uint16_t *d_txn_sz, const fdgpu_frag_ex_t *d_fx, const uint8_t *d_txn_out,
                                    int8_t *d_codes, uint8_t *d_trailers, hipStream_t stream);
/* fdgpu_submit_frags_io's kernels, each on at most FDGPU_IO_BLOCKS blocks
   whose waves stride over groups of 64 frags.  Ingest: per group, the wave
   reads the 64 records and payload addresses (one coalesced read of each over
   the bus), copies the group's payloads (16-B units, flattened over the
   group, four loads in flight per lane) from host memory (d_src[i], the
   registered region's device-side address) to d_arena + d_fx[i].off; with
   d_chk (n pairs {mcache line address, seq}, line 0: none) each line is
   re-read once the payload loads have returned, and a republished one marks
   the kept record FDGPU_FX_LAPPED; then lane i parses frag i (fd_txn_parse)
   and the wave takes its descriptor slots with one atomic add on *d_n_sig,
   which must be zero at the start (the finish kernel of the slot's previous
   gathered batch clears it: d_zero_next).  Finish: per group, lane i writes
   frag i's code, dedup tag and out size, then the wave assembles the group's
   out frags at d_out + d_fx[i].tr_off ([payload][pad][fd_txn_t][u16 sz]) in
   16-B stores. */
#define FDGPU_FX_LAPPED 0x80000000u     /* in fdgpu_frag_ex_t.tr_cap (out_cap <= 0xFFFF) */
/* DMA gather (d_rtab != NULL): the payloads already lie in the batch arena
   (the DMA engines copied the batch's source ranges there); a record's sz
   carries its range (bits 16..23) and off its offset in that range, and the
   ingest kernel only resolves off = d_rtab[range] + off */
#define FDGPU_IO_RANGES_MAX 255u
uint64_t   fdgpu_frag_fp_bound(uint32_t sz);
hipError_t fdgpu_launch_frag_ingest_io(const uint64_t *d_src, const fdgpu_frag_ex_t *d_fx, const uint64_t *d_chk,
                                       const uint64_t *d_rtab, uint32_t n, uint8_t *d_arena,
                                       fdgpu_frag_ex_t *d_fx_dev, uint8_t *d_txn_out, uint16_t *d_txn_sz,
                                       fdgpu_sig_desc_t *d_sigs, fdgpu_txn_desc_t *d_tds, uint32_t *d_n_sig,
                                       uint32_t *d_zero_word, hipStream_t stream);
hipError_t fdgpu_launch_frag_finish_io(const fdgpu_txn_desc_t *d_tds, uint32_t n, const int8_t *d_sig_codes,
                                       const uint16_t *d_txn_sz, const fdgpu_frag_ex_t *d_fx, const uint8_t *d_txn_out,
                                       const uint8_t *d_arena, uint64_t hash_seed, uint8_t *d_out, int8_t *d_codes,
                                       uint64_t *d_tags, uint16_t *d_out_szs, uint32_t *d_zero_next,
                                       hipStream_t stream);
hipError_t fdgpu_launch_test_hs_split(const uint32_t *d_in, uint32_t *d_out, uint32_t n, hipStream_t stream);

#ifdef __cplusplus
}
#endif
