/* fdgpu_kernels.hip -- MI355X (gfx950) kernels of the batched Ed25519
   verify engine.  One signature per lane, 256-thread workgroups; integer /
   bignum work only (no MFMA).  Per batch, on one stream:

   fdgpu_verify_hs_kernel  everything: S < L,
       k = SHA-512(R||A||M) mod L, decode A and R (decode2's rules and code
       order) with their small-order tests and the per-lane tables
       {O, -A, .., -8A}, {O, -R, .., -8R}; the lattice split of k into two
       ~128-bit scalars u = v k (mod 8L) (fdgpu_lattice.h); [w]B (w = v S
       mod L) by the fixed-base comb; [u](+-A) + [v](+-R) on one shared,
       divergence-free signed radix-16 chain with the table entries staged
       through LDS by LDS-DMA; the projective check against -[w]B.
   fdgpu_full_kernel       the rare lanes whose split failed: the full-length
       [S]B + [k](-A) chain, compared with the decoded R.
   fdgpu_key_dedup_kernel, fdgpu_key_table_kernel  (FDGPU_FLAG_KCACHE) one A
       decode + table per distinct public key, read in place by
       fdgpu_verify_hs_kernel<true> and the fallback kernel.
   fdgpu_combine_kernel    per transaction, batch_single_msg first-error
       semantics (fd_ed25519_user.c:232-310), plus a ballot-compacted
       accept bitmap.
   fdgpu_frag_* / fdgpu_scan_*  GPU-side ingest of raw payloads: fd_txn_parse
       (fdt_parse.h), the signature-count scan, the descriptor expansion.
   fdgpu_bcomb_*           build the comb tables at engine open.
   fdgpu_test_*            per-stage diagnostics for the parity tests. */
#include <hip/hip_runtime.h>

#include "fdgpu_ge.h"
#include "fdgpu_internal.h"
#include "fdgpu_sc.h"
#include "fdgpu_sha512.h"
#include "fdgpu_lattice.h"
#include "fdgpu_stamps.h"
#include "fdt_hash.h"
#include "fdt_parse.h"

using namespace fdgpu;

#ifndef FDGPU_VERIFY_WAVES
#define FDGPU_VERIFY_WAVES 2  /* waves per SIMD of the verify kernel: decode/pow chains want ~190 VGPRs */
#endif
/* A/B build switches.  The shipped library is built with every one at the
   default below; fdgpu_build_info() reports them and smoke() / bench.py
   refuse a library built otherwise (unless told it is an A/B build).
     FDGPU_TAB_STORE_NT   non-temporal stores of the chain tables
     FDGPU_TAB_LOAD_CPOL  cache-policy bits of the chain's LDS-DMA table loads
     FDGPU_WS_SLOT        chain tables in a per-device pool indexed by resident
                          block slot instead of by signature */
#ifndef FDGPU_TAB_STORE_NT
#define FDGPU_TAB_STORE_NT 0
#endif
#ifndef FDGPU_TAB_LOAD_CPOL
#define FDGPU_TAB_LOAD_CPOL 0
#endif
#ifndef FDGPU_WS_SLOT
#define FDGPU_WS_SLOT 0
#endif
#define FDGPU_WS_SLOTS 4096u        /* wave slots of the pool (>= the 2,048 verify waves a device keeps resident) */

namespace {

FDG_DEV void load32(uint32_t (&w)[8], const uint8_t *p) {
  /* 32-byte field (any 4-byte alignment in practice; use dword loads) */
  const uint32_t *q = (const uint32_t *)p;
  if (((uintptr_t)p & 3u) == 0) {
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = q[i];
  } else {
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = load_u32_unaligned(p + 4 * i);
  }
}

FDG_DEV void niels_store(uint32_t *dst, const fe &ypx, const fe &ymx, const fe &xy2d) {
#pragma unroll
  for (int i = 0; i < 10; i++) { dst[i] = ypx.v[i]; dst[10 + i] = ymx.v[i]; dst[20 + i] = xy2d.v[i]; }
  dst[30] = 0; dst[31] = 0;
}

/* ---- fixed-base comb tables ----
   table i, entry j = j * 2^(W i) B as affine niels (y+x, y-x, 2dxy),
   canonical limbs, word offset ((i * ENTRIES) + j) * STRIDE. */

constexpr uint32_t BC_W = FDGPU_BCOMB_BITS, BC_NDIG = FDGPU_BCOMB_NDIG, BC_ENT = FDGPU_BCOMB_ENTRIES;
constexpr uint32_t BC_CHUNKS = (BC_ENT + FDGPU_BCOMB_CHUNK - 1) / FDGPU_BCOMB_CHUNK;

/* bases[i] = 2^(W i) B (p3, 40 words), one lane per table */
__global__ void fdgpu_bcomb_base_kernel(uint32_t *bases) {
  const uint32_t i = threadIdx.x;
  if (i >= BC_NDIG) return;
  constexpr uint32_t BX[10] = FDGPU_FE_BX, BY[10] = FDGPU_FE_BY, BT[10] = FDGPU_FE_BT;
  ge_p3 P; fe_set(P.X, BX); fe_set(P.Y, BY); fe_1(P.Z); fe_set(P.T, BT);
  ge_p1p1 t;
  for (uint32_t n = 0; n < BC_W * i; n++) {
    ge_p2 a; ge_p3_to_p2(a, P); ge_dbl(t, a); ge_p1p1_to_p3(P, t);
  }
  uint32_t *o = bases + 40 * i;
#pragma unroll
  for (int w = 0; w < 10; w++) { o[w] = P.X.v[w]; o[10 + w] = P.Y.v[w]; o[20 + w] = P.Z.v[w]; o[30 + w] = P.T.v[w]; }
}

/* One lane per (table, chunk of 64 entries): j0 * base by double-and-add,
   then 63 consecutive additions, then one inversion for the whole chunk
   (Montgomery's trick over the Z coordinates, prefix products in scratch). */
__global__ void __launch_bounds__(64) fdgpu_bcomb_fill_kernel(const uint32_t *bases, uint32_t *tab,
                                                              uint32_t *scratch) {
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= BC_NDIG * BC_CHUNKS) return;
  const uint32_t ti = lane / BC_CHUNKS, j0 = (lane % BC_CHUNKS) * FDGPU_BCOMB_CHUNK;
  const uint32_t cnt = min(FDGPU_BCOMB_CHUNK, BC_ENT - j0);
  ge_p3 base;
  const uint32_t *b = bases + 40 * ti;
#pragma unroll
  for (int w = 0; w < 10; w++) { base.X.v[w] = b[w]; base.Y.v[w] = b[10 + w]; base.Z.v[w] = b[20 + w]; base.T.v[w] = b[30 + w]; }
  ge_cached bc; ge_p3_to_cached(bc, base);
  ge_p3 P; ge_p3_0(P);
  ge_p1p1 t;
  for (int bit = (int)BC_W - 1; bit >= 0; bit--) {                   /* j0 < 2^(W-1) + 1 */
    ge_p2 a; ge_p3_to_p2(a, P); ge_dbl(t, a); ge_p1p1_to_p3(P, t);
    if ((j0 >> bit) & 1u) { ge_add_cached(t, P, bc, false); ge_p1p1_to_p3(P, t); }
  }
  uint32_t *pre = scratch + (size_t)lane * FDGPU_BCOMB_CHUNK * 10;
  uint32_t *ent0 = tab + ((size_t)ti * BC_ENT + j0) * FDGPU_BCOMB_STRIDE;
  fe acc; fe_1(acc);
  for (uint32_t k = 0; k < cnt; k++) {
    uint32_t *e = ent0 + (size_t)k * FDGPU_BCOMB_STRIDE;
#pragma unroll
    for (int w = 0; w < 10; w++) { e[w] = P.X.v[w]; e[10 + w] = P.Y.v[w]; e[20 + w] = P.Z.v[w]; }
    fe_mul(acc, acc, P.Z);
#pragma unroll
    for (int w = 0; w < 10; w++) pre[10 * k + w] = acc.v[w];
    ge_add_cached(t, P, bc, false); ge_p1p1_to_p3(P, t);
  }
  fe inv; fe_invert(inv, acc);
  constexpr uint32_t D2[10] = FDGPU_FE_D2;
  fe d2; fe_set(d2, D2);
  for (int k = (int)cnt - 1; k >= 0; k--) {
    uint32_t *e = ent0 + (size_t)k * FDGPU_BCOMB_STRIDE;
    fe X, Y, Z, zi;
#pragma unroll
    for (int w = 0; w < 10; w++) { X.v[w] = e[w]; Y.v[w] = e[10 + w]; Z.v[w] = e[20 + w]; }
    if (k > 0) {
      fe pk;
#pragma unroll
      for (int w = 0; w < 10; w++) pk.v[w] = pre[10 * (k - 1) + w];
      fe_mul(zi, inv, pk);
    } else {
      zi = inv;
    }
    fe_mul(inv, inv, Z);
    fe x, y, xy, ypx, ymx, xy2d;
    fe_mul(x, X, zi); fe_mul(y, Y, zi);
    fe_add(ypx, y, x); fe_canon(ypx);
    fe_sub(ymx, y, x); fe_canon(ymx);
    fe_mul(xy, x, y); fe_mul(xy2d, xy, d2); fe_canon(xy2d);
    niels_store(e, ypx, ymx, xy2d);
  }
}

/* ---- per-lane tables in the global workspace ----
   layout: lane-contiguous, ws[i * FDGPU_WS_LANE_WORDS + entry * 40 + word]
   for signature i: a lane's entry is 160 contiguous bytes (32-B aligned),
   read whole with ten 16-B loads, so a wave's table read touches ~2 cache
   lines per lane and uses every byte it fetches (fdgpu_internal.h lists the
   entries). */

/* Stored word order of a cached entry: Y+X and Y-X
   interleaved by pairs in the first five 16-B chunks -- chunk k = (Y+X
   limbs 2k, 2k+1, Y-X limbs 2k, 2k+1) -- then 2Z and 2dT as they are.  A
   chain addition of -P reads Y+X and Y-X swapped: with pairs the swap is a
   per-lane 8-B offset of two ds_read_b64 (unstage_entry_signed) instead of
   20 per-word selects.  atab_store / atab_load convert, so every other
   reader sees the canonical order (Y+X, Y-X, 2Z, 2dT). */
__host__ __device__ constexpr int atab_pos(int w) {
  return w >= 20 ? w : w < 10 ? 4 * (w / 2) + (w % 2) : 4 * ((w - 10) / 2) + 2 + (w % 2);
}

/* A table's entry 0 -- the identity in cached form (Y+X = Y-X = 1, 2Z = 2,
   2dT = 0) in the stored word order -- is this one constant for every lane
   and table: digit-0 lookups read it (an L2 hit), and a lane's workspace
   holds only entries 1..8 of its tables (2880 B per signature instead of
   3200, a smaller footprint in the caches the table reads hit). */
struct alignas(16) tab_ident_t { uint32_t w[FDGPU_ATAB_WORDS]; };
__device__ const tab_ident_t g_tab_ident = {{1u, 0u, 1u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 2u}};
static_assert(atab_pos(0) == 0 && atab_pos(10) == 2 && atab_pos(20) == 20, "identity entry's stored order");

/* Entry |e| of a table whose (virtual) base is `tab` (entry k at tab + 40 k
   for k >= 1; see tab_a / tab_r): the shared identity for e == 0. */
FDG_DEV const uint32_t *tab_entry(const uint32_t *tab, int e) {
  return e ? tab + (uint32_t)(e < 0 ? -e : e) * FDGPU_ATAB_WORDS : g_tab_ident.w;
}
/* virtual bases of a lane's -A and -R tables: stored entry 1 sits at the
   table's first workspace entry */
FDG_DEV uint32_t *tab_a(uint32_t *wsl) { return wsl - FDGPU_ATAB_WORDS; }
FDG_DEV const uint32_t *tab_a(const uint32_t *wsl) { return wsl - FDGPU_ATAB_WORDS; }
FDG_DEV uint32_t *tab_r(uint32_t *wsl) { return wsl + (FDGPU_WS_RTAB - 1u) * FDGPU_ATAB_WORDS; }

FDG_DEV void atab_store(uint32_t *wsl, uint32_t entry, const ge_cached &c) {
  uint4 *p = (uint4 *)(wsl + entry * FDGPU_ATAB_WORDS);
  uint32_t w[40], o[40];
#pragma unroll
  for (int i = 0; i < 10; i++) { w[i] = c.YpX.v[i]; w[10 + i] = c.YmX.v[i]; w[20 + i] = c.Z2.v[i]; w[30 + i] = c.T2d.v[i]; }
#pragma unroll
  for (int i = 0; i < 40; i++) o[atab_pos(i)] = w[i];
#pragma unroll
  for (int q = 0; q < 10; q++) {
#if FDGPU_TAB_STORE_NT
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = {o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]};
    __builtin_nontemporal_store(v, (u32x4 *)(p + q));
#else
    p[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
#endif
  }
}
FDG_DEV int sext4(uint32_t x) { return ((int)(x << 28)) >> 28; }

#define KD_WORDS 8        /* 64 signed radix-16 digits of k, one per nibble */

FDG_DEV void atab_load(uint32_t (&q)[40], const uint32_t *wsl, int e) {
  const uint4 *ent = (const uint4 *)tab_entry(wsl, e);
  uint32_t o[40];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const uint4 v = ent[i];
    o[4 * i] = v.x; o[4 * i + 1] = v.y; o[4 * i + 2] = v.z; o[4 * i + 3] = v.w;
  }
#pragma unroll
  for (int i = 0; i < 40; i++) q[i] = o[atab_pos(i)];
}

/* shift a 256-bit little-endian word vector left by 4 bits */
FDG_DEV void shl4(uint32_t (&w)[8]) {
#pragma unroll
  for (int i = 7; i > 0; i--) w[i] = (w[i] << 4) | (w[i - 1] >> 28);
  w[0] <<= 4;
}

/* R' = [k](-A) + [S]B with [S]B precomputed by the
   comb in pass 1 and parked (cached form) in workspace entry 10.  The chain
   only serves k: 64 windows of 4 doublings + one A-table addition; the last
   window's sum is converted to p3 and the parked [S]B added. */
FDG_DEV void dsm_k(ge_p2 &acc2, uint32_t (&kd)[KD_WORDS], const uint32_t *wsl, uint32_t sb_entry = FDGPU_WS_SB,
                   const uint32_t *ta = nullptr) {
  if (!ta) ta = tab_a(wsl);               /* the -A table: own workspace, or the key cache's */
  ge_p3 acc3;
  ge_p1p1 t;
  uint32_t q[40];
  /* the top window would double the identity four times and then add its
     entry: start from the entry itself (Horner's first step) */
  {
    const int e = sext4(kd[7] >> 28);
    shl4(kd);
    atab_load(q, ta, e);
    ge_cached_regs_to_p2(acc2, q, e < 0);
  }
#pragma unroll 1
  for (int j = 62; j >= 0; j--) {
    const int e = sext4(kd[7] >> 28);
    shl4(kd);
    atab_load(q, ta, e);
#pragma unroll 1
    for (int r = 0; r < 4; r++) {
      ge_dbl(t, acc2);
      ge_p1p1_to_p2(acc2, t);
    }
    acc3.X = acc2.X; acc3.Y = acc2.Y; acc3.Z = acc2.Z; fe_mul(acc3.T, t.X, t.Y);
    ge_add_cached_regs(t, acc3, q, e < 0);
    if (j == 0) break;
    ge_p1p1_to_p2(acc2, t);
  }
  /* + [S]B (parked cached form) */
  ge_p1p1_to_p3(acc3, t);
  uint32_t qs[40];
  atab_load(qs, wsl, (int)sb_entry);
  ge_add_cached_regs(t, acc3, qs, false);
  ge_p1p1_to_p2(acc2, t);
}

/* [S]B by the fixed-base comb: S (< L, or 0 for rejected lanes) in signed
   radix 2^W; one mixed addition per digit from table i; each entry (one
   128-B line, random across the 67-MB table) is loaded one digit ahead of
   its use so the load latency hides behind the previous addition.  [lo, hi)
   sums only the digits of tables lo..hi-1 (the two-lane kernel splits the
   comb over a pair: 2 + 2 x 7 additions instead of 15 per lane). */
FDG_DEV void comb_sb(ge_p3 &acc, const uint32_t (&S)[8], const uint32_t *__restrict__ btab, uint32_t lo = 0,
                     uint32_t hi = BC_NDIG) {
  constexpr int NW = COMB_WORDS(BC_W, BC_NDIG), SLOT = COMB_SLOT(BC_W);
  uint32_t dg[NW];
  sc_recode_comb<(int)BC_W, (int)BC_NDIG>(dg, S);
  auto next_digit = [&dg]() {
    const int d = SLOT == 16 ? (int)(int16_t)(dg[0] & 0xffffu) : (int)dg[0];
#pragma unroll
    for (int i = 0; i < NW - 1; i++) dg[i] = SLOT == 16 ? (dg[i] >> 16) | (dg[i + 1] << 16) : dg[i + 1];
    dg[NW - 1] = SLOT == 16 ? dg[NW - 1] >> 16 : 0u;
    return d;
  };
  auto load_entry = [btab](uint32_t (&q)[32], uint32_t ti, int d) {
    const uint4 *ent = (const uint4 *)(btab + ((size_t)ti * BC_ENT + (uint32_t)(d < 0 ? -d : d)) * FDGPU_BCOMB_STRIDE);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint4 v = ent[i];
      q[4 * i] = v.x; q[4 * i + 1] = v.y; q[4 * i + 2] = v.z; q[4 * i + 3] = v.w;
    }
  };
  uint32_t qa[32], qb[32];
#pragma unroll 1
  for (uint32_t i = 0; i < lo; i++) (void)next_digit();
  int d = next_digit();
  load_entry(qa, lo, d);
  /* the first digit's entry is the starting point (no addition to O) */
  {
    const int dn = next_digit();
    load_entry(qb, lo + 1, dn);
    ge_niels_regs_to_p3(acc, qa, d < 0);
#pragma unroll
    for (int w = 0; w < 32; w++) qa[w] = qb[w];
    d = dn;
  }
  ge_p1p1 t;
#pragma unroll 1
  for (uint32_t i = lo + 1; i < hi; i++) {
    const int dn = next_digit();
    if (i + 1 < hi) load_entry(qb, i + 1, dn);
    ge_add_niels_regs(t, acc, qa, d < 0);
    ge_p1p1_to_p3(acc, t);
#pragma unroll
    for (int w = 0; w < 32; w++) qa[w] = qb[w];
    d = dn;
  }
}

/* Build this lane's table {-A, -2A, ..., -8A} (cached form; O is the
   shared g_tab_ident) in the workspace.  Even multiples by doubling the stored half (4S + 4M) instead
   of adding -A (8M): 3 = 2 + 1, 4 = 2*2, 5 = 4 + 1, 6 = 2*3, 7 = 6 + 1,
   8 = 2*4. */
FDG_DEV void atab_build(uint32_t *wsl, const ge_p3 &An) {   /* wsl: the table's virtual base (tab_a / tab_r) */
  ge_cached c;
  ge_p3_to_cached(c, An); atab_store(wsl, 1, c);
  ge_p1p1 t; ge_p2 a2; ge_p3 P;
  ge_p3_to_p2(a2, An); ge_dbl(t, a2); ge_p1p1_to_p3(P, t);          /* 2(-A) */
  ge_p3_to_cached(c, P); atab_store(wsl, 2, c);
  const uint32_t *ent1 = wsl + 1u * FDGPU_ATAB_WORDS;
  auto ld1 = [ent1](int cc, int w) { return ent1[atab_pos(10 * cc + w)]; };
#pragma unroll 1
  for (uint32_t e = 3; e < FDGPU_ATAB_ENTRIES; e++) {
    if (e & 1u) {
      ge_add_cached_ld(t, P, ld1, false);
    } else {
      uint32_t q[40];
      atab_load(q, wsl, (int)(e >> 1));
      ge_cached_regs_to_p2(a2, q, false);
      ge_dbl(t, a2);
    }
    ge_p1p1_to_p3(P, t);
    ge_p3_to_cached(c, P); atab_store(wsl, e, c);
  }
}

FDG_DEV uint32_t *lane_ws(uint32_t *ws, uint32_t i) {
  return ws + (size_t)i * FDGPU_WS_LANE_WORDS;
}

/* FDGPU_WS_SLOT: the slot pool follows the comb tables in the per-device
   allocation (fdgpu_btab_bytes): a bitmap of FDGPU_WS_SLOTS bits (512 B),
   then one 64-lane workspace per slot.  A wave claims a free slot at its
   start and frees it at its end, so at most the device's resident verify
   waves' tables are live, and a new wave rewrites lines an earlier wave used
   instead of allocating fresh ones.  No wait: a wave that finds no free slot
   (never, with more slots than resident waves) keeps its per-signature
   workspace.  Per wave, not per block: a block-wide slot index in LDS would
   push the block past 80 KB, and two no longer fit a CU. */
#define WS_SLOT_NONE 0xFFFFFFFFu
#define BTAB_WORDS ((size_t)BC_NDIG * BC_ENT * FDGPU_BCOMB_STRIDE)
FDG_DEV uint32_t *ws_slot_bitmap(const uint32_t *btab) { return const_cast<uint32_t *>(btab) + BTAB_WORDS; }
FDG_DEV uint32_t *ws_slot_lanes(const uint32_t *btab, uint32_t slot) {
  return ws_slot_bitmap(btab) + FDGPU_WS_SLOTS / 32u + (size_t)slot * 64u * FDGPU_WS_LANE_WORDS;
}
FDG_DEV uint32_t ws_slot_claim(uint32_t *bm, uint32_t seed) {
  constexpr uint32_t NW = FDGPU_WS_SLOTS / 32u;
  for (uint32_t t = 0; t < 2u * NW; t++) {
    const uint32_t w = (seed + t) % NW;
    uint32_t v = __hip_atomic_load(bm + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (v != 0xFFFFFFFFu) {
      const uint32_t b = (uint32_t)__builtin_ctz(~v);
      const uint32_t old = atomicOr(bm + w, 1u << b);
      if (!(old & (1u << b))) return w * 32u + b;
      v = old | (1u << b);
    }
  }
  return WS_SLOT_NONE;
}
FDG_DEV void ws_slot_release(uint32_t *bm, uint32_t slot) { atomicAnd(bm + slot / 32u, ~(1u << (slot % 32u))); }

/* Output slot of lane i: signatures may be verified in an order grouped by
   SHA-512 block count (perm[i] = the signature's index in the caller's
   order); codes are always written in the caller's order. */
FDG_DEV uint32_t out_idx(const uint32_t *__restrict__ perm, uint32_t i) { return perm ? perm[i] : i; }

/* ---------------- half-size verify ----------------
   fdgpu_lattice.h: with u = v k (mod 8L), v odd and |u|, |v| < 2^159,
   [S]B - [k]A == R  <=>  [w]B - [u]A - [v]R == O  (w = v S mod L), decided
   with ~132 doublings instead of ~252.  Per lane:
     pass 1   S < L, k = SHA-512(R||A||M) mod L, decode A and R (the
              reference's decode2, both codes settled here in the
              reference's order), the tables {O, -A, .., -8A} and
              {O, -R, .., -8R};
     split    (u, v) = hs_split(k);  w = v S mod L;  [w]B by the comb;
     chain    [|u|](+-A table) + [|v|](+-R table) over the wave's longest
              digit string (signed radix 16: 4 doublings + 2 additions per
              window, every lane at the same positions);
     check    chain == -[w]B, projectively (4 products).
   A lane whose split fails (hs_split_t.ok == false) keeps k's digits and
   [S]B and is finished by fdgpu_full_kernel with the full-length chain. */

/* park words (entry FDGPU_WS_PARK) */
#define HPARK_KD 0        /* 8 words: radix-16 digits of k (full-path lanes) */
#define HPARK_CODE 30     /* pass-1 code */
/* (decoded R is not parked: fdgpu_full_kernel compares with the -R table's
   entry 1, projectively, so a half-size lane never writes this entry) */
static_assert(HPARK_KD + KD_WORDS <= HPARK_CODE && HPARK_CODE < (int)FDGPU_ATAB_WORDS, "park layout");

/* Signed radix-16 digits of a magnitude m < 2^160 (5 limbs): 40 nibbles in
   [-8, 7] (two's complement, digit i at bits 4(i%8) of word i/8); nd = the
   number of digits up to the highest nonzero one (41 if a carry is left). */
FDG_DEV void recode16_160(uint32_t (&out)[5], uint32_t &nd, const uint32_t (&m)[5]) {
  uint32_t carry = 0;
  nd = 0;
#pragma unroll
  for (int w = 0; w < 5; w++) {
    uint32_t o = 0;
#pragma unroll
    for (int n = 0; n < 8; n++) {
      uint32_t e = ((m[w] >> (4 * n)) & 15u) + carry;
      carry = e >= 8u;
      e = (e - (carry << 4)) & 15u;
      o |= e << (4 * n);
      nd = e ? (uint32_t)(8 * w + n + 1) : nd;
    }
    out[w] = o;
  }
  nd = carry ? 41u : nd;
}

FDG_DEV void shl4_5(uint32_t (&w)[5]) {
#pragma unroll
  for (int i = 4; i > 0; i--) w[i] = (w[i] << 4) | (w[i - 1] >> 28);
  w[0] <<= 4;
}

/* w = v S mod L for |v| < 2^160 (5 limbs), S < L (8 limbs); negated mod L
   when v < 0 */
FDG_DEV void hs_wscalar(uint32_t (&w)[8], const uint32_t (&v)[5], bool v_neg, const uint32_t (&S)[8]) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint64_t t = (uint64_t)v[i] * S[j] + x[i + j] + c;
      x[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    x[i + 8] = (uint32_t)c;
  }
  uint32_t r[8];
  sc_reduce512(r, x);
  constexpr uint32_t L[8] = FDGPU_SC_L;
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) nz |= r[i];
  const bool flip = v_neg && nz != 0;
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {                 /* L - r */
    const uint64_t d = (uint64_t)L[i] - r[i] - bw;
    w[i] = flip ? (uint32_t)d : r[i];
    bw = (uint32_t)(d >> 63);
  }
}

/* Table entries of the chain are staged through LDS by LDS-DMA
   (global_load_lds_dwordx4: no VGPR destination), issued at the start of a
   window and read back after its doublings, so no 40-word entry stays live
   in VGPRs across the doublings.  One wave-instruction moves 16 B for each
   of the 64 lanes into 1 KiB of LDS (wave-uniform base + 16 B x lane).
   Both entries of a window go through LDS (2 x 10 KiB per wave). */
typedef __attribute__((address_space(3))) void lds_void_t;

FDG_DEV void stage_entry(uint32_t *lds_wave, const uint32_t *tab, int e) {
  const uint32_t *src = tab_entry(tab, e);
  constexpr int NCH = 10;
#pragma unroll
  for (int c = 0; c < NCH; c++)
    __builtin_amdgcn_global_load_lds((const void *)(src + 4 * c), (lds_void_t *)(lds_wave + 256 * c), 16, 0,
                                     FDGPU_TAB_LOAD_CPOL);
}

/* The staged entry of a signed digit: q[0..9] = Y+X of the digit's point
   (Y-X of the table's -kP when neg), q[10..19] the other, 2Z, 2dT as stored
   (2dT still to be negated when neg).  With the pair-interleaved entries the
   swap is the 8-B offset of two ds_read_b64 per pair chunk. */
FDG_DEV void unstage_entry_signed(uint32_t (&q)[40], const uint32_t *lds_wave, bool neg) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t *a = lds_wave + 4 * lane + (neg ? 2u : 0u), *b = lds_wave + 4 * lane + (neg ? 0u : 2u);
#pragma unroll
  for (int c = 0; c < 5; c++) {
    const uint2 x = *(const uint2 *)(a + 256 * c), y = *(const uint2 *)(b + 256 * c);
    q[2 * c] = x.x; q[2 * c + 1] = x.y; q[10 + 2 * c] = y.x; q[10 + 2 * c + 1] = y.y;
  }
#pragma unroll
  for (int c = 5; c < 10; c++) {
    const uint4 v = *(const uint4 *)(lds_wave + 256 * c + 4 * lane);
    q[4 * c] = v.x; q[4 * c + 1] = v.y; q[4 * c + 2] = v.z; q[4 * c + 3] = v.w;
  }
}

/* [|u|](T_A) + [|v|](T_R), digit strings pre-shifted so that digit nwin-1
   sits in the top nibble; u_neg / v_neg flip every digit's sign (the tables
   hold -A, -R).  Leaves the completed sum of the last addition in t. */
FDG_DEV void hs_chain(ge_p1p1 &t, uint32_t (&ud)[5], uint32_t (&vd)[5], bool u_neg, bool v_neg, uint32_t nwin,
                      const uint32_t *wsl, const uint32_t *ta) {
  const uint32_t *tr = tab_r(const_cast<uint32_t *>(wsl));
  __shared__ uint32_t s_stage[FDGPU_BLOCK / 64][2][10 * 256];
  uint32_t *st_r = &s_stage[threadIdx.x >> 6][0][0];
  uint32_t *st_a = &s_stage[threadIdx.x >> 6][1][0];
  ge_p2 acc2;
  ge_p3 acc3;
  uint32_t q[40];
  {                                             /* top window: O + T_A[du] + T_R[dv] */
    const int du = sext4(ud[4] >> 28), dv = sext4(vd[4] >> 28);
    shl4_5(ud); shl4_5(vd);
    /* the entry as a p3 point needs T = XY/Z (its 2dT would need 1/d): add
       it to the identity instead */
    atab_load(q, ta, du);
    ge_p3_0(acc3);
    ge_add_cached_regs(t, acc3, q, (du < 0) != u_neg);
    ge_p1p1_to_p3(acc3, t);
    atab_load(q, tr, dv);
    ge_add_cached_regs(t, acc3, q, (dv < 0) != v_neg);
  }
#pragma unroll 1
  for (uint32_t j = 1; j < nwin; j++) {
    ge_p1p1_to_p2(acc2, t);
    const int du = sext4(ud[4] >> 28), dv = sext4(vd[4] >> 28);
    shl4_5(ud); shl4_5(vd);
    stage_entry(st_a, ta, du);
    stage_entry(st_r, tr, dv);
#pragma unroll 1
    for (int r = 0; r < 4; r++) {
      ge_dbl(t, acc2);
      ge_p1p1_to_p2(acc2, t);
    }
    acc3.X = acc2.X; acc3.Y = acc2.Y; acc3.Z = acc2.Z; fe_mul(acc3.T, t.X, t.Y);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   /* the window's LDS-DMA has landed */
    unstage_entry_signed(q, st_a, (du < 0) != u_neg);
    ge_add_cached_regs_swapped(t, acc3, q, (du < 0) != u_neg);
    ge_p1p1_to_p3(acc3, t);
    unstage_entry_signed(q, st_r, (dv < 0) != v_neg);
    ge_add_cached_regs_swapped(t, acc3, q, (dv < 0) != v_neg);
  }
}

/* The verify kernel of the half-size path; codes of lanes it settles are
   written here, lanes whose split failed are queued for fdgpu_full_kernel.
   The body takes its block index: the merged launch (fdgpu_verify_hs_multi_kernel)
   runs it for the batch blockIdx.y names.  PH (prehashed, the synchronous
   API's messages too large for one arena): the descriptor's msg_off holds
   the lane's SHA-512(R || A || M) state words, hashed beforehand in pieces
   by fdgpu_sha512_stream_kernel; the product instantiations have PH false. */
template <bool KC, bool PH = false>
FDG_DEV void verify_hs_body(const uint8_t *__restrict__ arena, const fdgpu_sig_desc_t *__restrict__ sigs, uint32_t n_sig_arg,
                            const uint32_t *__restrict__ n_sig_dev, const uint32_t *__restrict__ btab,
                            uint32_t *__restrict__ ws, const uint32_t *__restrict__ perm, int8_t *__restrict__ codes,
                            uint32_t *__restrict__ queue, uint32_t *__restrict__ queue_cnt, uint32_t flags,
                            const uint32_t *__restrict__ key_of, const uint32_t *__restrict__ kverd, uint32_t bx) {
  /* n_sig_dev: the count is produced on the device (GPU-side ingest) and the
     grid covers an upper bound; blocks past it leave at once */
  const uint32_t n_sig = n_sig_dev ? *n_sig_dev : n_sig_arg;
  if (bx * blockDim.x >= n_sig) return;
  const uint32_t i = bx * blockDim.x + threadIdx.x;
  const bool active = i < n_sig;
  const bool ref_map = (flags & FDGPU_FLAG_REF_MAP) != 0;
  const fdgpu_sig_desc_t d = sigs[active ? i : n_sig - 1];
  uint32_t nb = sha512_hram_blocks(d.msg_sz);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) nb = max(nb, (uint32_t)__shfl_xor((int)nb, off));
  uint32_t *wsl = lane_ws(ws, i);
#if FDGPU_WS_SLOT
  uint32_t w_slot = WS_SLOT_NONE;
  if (!KC) {
    if ((threadIdx.x & 63u) == 0) w_slot = ws_slot_claim(ws_slot_bitmap(btab), (bx * 4u + (threadIdx.x >> 6)) * 7u);
    w_slot = __builtin_amdgcn_readfirstlane(w_slot);
    if (w_slot != WS_SLOT_NONE) wsl = ws_slot_lanes(btab, w_slot) + (size_t)(threadIdx.x & 63u) * FDGPU_WS_LANE_WORDS;
  }
#endif
  uint32_t *park = wsl + FDGPU_WS_PARK * FDGPU_ATAB_WORDS;
  const uint32_t *ta = tab_a(wsl);             /* this lane's -A table */
  FDGPU_STAMP(0);
  uint32_t Renc[8], Aenc[8];
  load32(Renc, arena + d.sig_off);
  load32(Aenc, arena + d.pub_off);
  /* k = SHA-512(R || A || M) mod L */
  uint32_t k[8];
  {
    uint64_t h[8];
    if (PH) {
#pragma unroll
      for (int j = 0; j < 8; j++) h[j] = ((const uint64_t *)(arena + d.msg_off))[j];
    } else {
      sha512_hram(h, Renc, Aenc, arena + d.msg_off, d.msg_sz, nb);
    }
    FDGPU_STAMP(1);
    uint32_t kx[16];
#pragma unroll
    for (int j = 0; j < 8; j++) { kx[2 * j] = bswap32((uint32_t)(h[j] >> 32)); kx[2 * j + 1] = bswap32((uint32_t)h[j]); }
    sc_reduce512(k, kx);
  }
  /* step 1: S < L (fd_ed25519_user.c:159-161) */
  uint32_t S[8];
  load32(S, arena + d.sig_off + 32);
  int code = sc_lt_L(S) ? 0 : -1;
#pragma unroll
  for (int j = 0; j < 8; j++) S[j] = code ? 0u : S[j];
  FDGPU_STAMP(2);
  /* step 2: decode A then R (decode2 reports A first), small-order tests,
     tables of -A and -R */
  {
    ge_p3 P, Pn;
    bool a_ok, a_small;
    if (KC) {
      /* key cache: the -A table was built once per distinct key by
         fdgpu_key_table_kernel in its representative lane's workspace, and
         the chain reads it there */
      const uint32_t di = active ? i : n_sig - 1u, r = key_of[di], vd = kverd[r];
      a_ok = (vd & 1u) != 0;
      a_small = (vd & 2u) != 0;
      ta = tab_a(lane_ws(ws, r));
    } else {
      a_ok = ge_decode(P, Aenc, ref_map);
      a_small = ge_is_small_order_affine(P);
      ge_p3_neg(Pn, P);
      atab_build(tab_a(wsl), Pn);
    }
    FDGPU_STAMP(3);
    const bool r_ok = ge_decode(P, Renc, ref_map);
    const bool r_small = ge_is_small_order_affine(P);
    ge_p3_neg(Pn, P);
    atab_build(tab_r(wsl), Pn);
    if (code == 0 && !a_ok) code = ref_map ? -2 : -1;
    if (code == 0 && !r_ok) code = -1;
    if (code == 0 && a_small) code = -2;                 /* fd_ed25519_user.c:194-199 */
    if (code == 0 && r_small) code = -1;
  }
  FDGPU_STAMP(4);
  const bool need = active && code == 0;
  /* split k (lanes already failed run no Euclid steps: k = 0) */
  hs_split_t hs;
  {
    uint32_t ke[8];
#pragma unroll
    for (int j = 0; j < 8; j++) ke[j] = need ? k[j] : 0u;
    hs_split(hs, ke);
  }
  uint32_t ud[5], vd[5], ndu = 0, ndv = 0;
  recode16_160(ud, ndu, hs.u);
  recode16_160(vd, ndv, hs.v);
  const uint32_t nd_lane = max(max(ndu, ndv), 1u);
  const bool full = need && (!hs.ok || nd_lane > HS_MAX_WIN || (flags & FDGPU_FLAG_KFULL));
  const bool half = need && !full;
  FDGPU_STAMP(5);
  /* [w]B (w = v S mod L), or [S]B for the full-length path; parked cached */
  {
    uint32_t w[8];
    hs_wscalar(w, hs.v, hs.v_neg, S);
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = half ? w[j] : S[j];
    ge_p3 WB;
    comb_sb(WB, w, btab);
    ge_cached c; ge_p3_to_cached(c, WB);
    atab_store(wsl, FDGPU_WS_SB, c);
  }
  if (full) {
    uint32_t kd[KD_WORDS];
    sc_recode16(kd, k);
#pragma unroll
    for (int j = 0; j < KD_WORDS; j++) park[HPARK_KD + j] = kd[j];
    park[HPARK_CODE] = 0u;
#if FDGPU_WS_SLOT
    /* fdgpu_full_kernel reads the lane's workspace by signature: a slot
       lane parks a copy of its tables, [S]B and k there */
    uint32_t *own = lane_ws(ws, i);
    if (own != wsl)
      for (uint32_t q = 0; q < FDGPU_WS_LANE_WORDS / 4u; q++) ((uint4 *)own)[q] = ((const uint4 *)wsl)[q];
#endif
  }
  FDGPU_STAMP(6);
  bool eq = false;
  if (__any(half)) {
    /* the wave's digit count; every lane runs it (shorter strings lead with zeros) */
    uint32_t nwin = half ? nd_lane : 1u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nwin = max(nwin, (uint32_t)__shfl_xor((int)nwin, off));
#pragma unroll 1
    for (uint32_t s = nwin; s < 40; s++) { shl4_5(ud); shl4_5(vd); }
    ge_p1p1 t;
    hs_chain(t, ud, vd, hs.u_neg, hs.v_neg, nwin, wsl, ta);
    /* chain == -[w]B:  x = X/Z = -(YpX - YmX)/Z2,  y = Y/T = (YpX + YmX)/Z2 */
    uint32_t q[40];
    atab_load(q, wsl, (int)FDGPU_WS_SB);
    fe ypx, ymx, z2, xw, yw, l1, l2;
#pragma unroll
    for (int j = 0; j < 10; j++) { ypx.v[j] = q[j]; ymx.v[j] = q[10 + j]; z2.v[j] = q[20 + j]; }
    fe_sub(xw, ypx, ymx);
    fe_add(yw, ypx, ymx);
    fe_mul(l1, t.X, z2);
    fe_mul(l2, t.Z, xw);
    fe_add(l1, l1, l2);
    const bool ex = fe_iszero(l1);
    fe_mul(l1, t.Y, z2);
    fe_mul(l2, t.T, yw);
    fe_sub(l1, l1, l2);
    eq = ex && fe_iszero(l1);
  }
  FDGPU_STAMP(7);
  if (active && !full) codes[out_idx(perm, i)] = (int8_t)(code ? code : (eq ? 0 : -3));
  {                                             /* queue the full-length lanes (rare) */
    const uint64_t m = __ballot(full);
    if (m) {
      const int lane = (int)(threadIdx.x & 63u);
      const int leader = __ffsll((long long)m) - 1;
      uint32_t base = 0;
      if (lane == leader) base = atomicAdd(queue_cnt, (uint32_t)__popcll(m));
      base = (uint32_t)__shfl((int)base, leader, 64);
      if (full) queue[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = i;
    }
  }
#if FDGPU_WS_SLOT
  if (!KC && w_slot != WS_SLOT_NONE) {          /* every access of the wave to its slot has completed: free it */
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63u) == 0) ws_slot_release(ws_slot_bitmap(btab), w_slot);
  }
#endif
}

template <bool KC, bool PH = false>
__global__ void __launch_bounds__(FDGPU_BLOCK, FDGPU_VERIFY_WAVES)
fdgpu_verify_hs_kernel(const uint8_t *__restrict__ arena, const fdgpu_sig_desc_t *__restrict__ sigs, uint32_t n_sig_arg,
                       const uint32_t *__restrict__ n_sig_dev, const uint32_t *__restrict__ btab,
                       uint32_t *__restrict__ ws, const uint32_t *__restrict__ perm, int8_t *__restrict__ codes,
                       uint32_t *__restrict__ queue, uint32_t *__restrict__ queue_cnt, uint32_t flags,
                       const uint32_t *__restrict__ key_of, const uint32_t *__restrict__ kverd) {
  verify_hs_body<KC, PH>(arena, sigs, n_sig_arg, n_sig_dev, btab, ws, perm, codes, queue, queue_cnt, flags, key_of,
                         kverd, blockIdx.x);
}

/* SHA-512(R_i || A_i || M) of one message shared by n <= 64 signatures (lane
   i: signature i), over blocks [blk0, blk0 + nblk) of the n streams, in a
   launch per piece of M: the synchronous API's messages too large for one
   arena.  state: n x 8 words (initialised by the launch with blk0 == 0),
   left as sha512_hram leaves its h.  mbuf holds M[m0, m0 + mlen): every
   message byte of the launch's blocks (the host's piece).  Block b of a
   stream is R || A || M[0, 64) for b = 0 and M[128 b - 64, 128 b + 64)
   after, padded past msg_sz and length-terminated as sha512_hram does;
   bytes are gathered one by one (a rare path, one wave). */
__global__ void __launch_bounds__(64) fdgpu_sha512_stream_kernel(const uint8_t *__restrict__ mbuf, uint64_t m0,
                                                                 uint64_t mlen, uint64_t msg_sz, uint64_t blk0,
                                                                 uint32_t nblk, const uint8_t *__restrict__ ra,
                                                                 uint64_t *__restrict__ state, uint32_t n) {
  const uint32_t i = threadIdx.x;
  if (i >= n) return;
  const uint64_t H0[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                          0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                          0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  uint64_t h[8];
  for (int j = 0; j < 8; j++) h[j] = blk0 ? state[8 * i + j] : H0[j];
  const uint64_t total = (64u + msg_sz + 16u) / 128u + 1u, bitlen = (64u + msg_sz) * 8u;
  for (uint64_t b = blk0; b < blk0 + nblk; b++) {
    uint64_t w[16];
    for (int t = 0; t < 16; t++) {
      uint64_t v = 0;
      for (int j = 0; j < 8; j++) {
        const uint64_t s = 128u * b + 8u * (uint64_t)t + (uint64_t)j;     /* position in R || A || M */
        uint32_t byte;
        if (s < 64u) {
          byte = ra[64u * i + s];
        } else {
          const uint64_t g = s - 64u;                                     /* position in M */
          byte = g < msg_sz ? (g >= m0 && g < m0 + mlen ? mbuf[g - m0] : 0u) : g == msg_sz ? 0x80u : 0u;
        }
        v = (v << 8) | byte;
      }
      w[t] = v;
    }
    if (b + 1 == total) { w[14] = 0; w[15] = bitlen; }
    sha512_compress(h, w);
  }
  for (int j = 0; j < 8; j++) state[8 * i + j] = h[j];
}

/* Several batches' verifies as ONE launch (FDGPU_FLAG_MERGE): block (x, y)
   is block x of batch y.  Concurrent 16 K-signature launches from separate
   streams share the CUs badly -- eight 8 K launches at once take 1.33 ms,
   one 64 K launch 0.85 ms (profiles/r04/conc_probe.jsonl) -- so an engine
   with several batches ready verifies them together. */
__global__ void __launch_bounds__(FDGPU_BLOCK, FDGPU_VERIFY_WAVES)
fdgpu_verify_hs_multi_kernel(const fdgpu_mbatch_t *__restrict__ mb, const uint32_t *__restrict__ btab, uint32_t flags) {
  const fdgpu_mbatch_t b = mb[blockIdx.y];
  if (blockIdx.x * blockDim.x >= b.bound) return;
  verify_hs_body<false>(b.arena, b.sigs, b.bound, b.n_sig, btab, b.ws, nullptr, b.codes, b.queue, b.cnt, flags, nullptr,
                        nullptr, blockIdx.x);
}

/* ---------------- two lanes per signature (FDGPU_FLAG_KPAIR) ----------------
   The same equation as fdgpu_verify_hs_kernel, with the work of one
   signature split over two adjacent lanes of a wave, for batches too small
   to fill the GPU's wave slots (a lone wave's lifetime is then the batch's
   latency).  Lane 2i (the A lane) decodes A and builds the -A table while
   lane 2i+1 (the R lane) decodes R and builds the -R table: one
   exponentiation per lane instead of two.  Each lane then runs a chain over
   its own half-size scalar -- [|u|](+-A) or [|v|](+-R), 4 doublings and ONE
   addition per window -- and the two sums are exchanged across the pair and
   added, so both lanes hold the complete [u](-A) + [v](-R) for the check
   against -[w]B.  SHA-512, the split and the comb run in both lanes (SIMT:
   it costs the wave the same time as running them in one).  Per signature
   the pair does ~1.4x the work of one lane; per wave it finishes ~30%
   sooner.  Lanes whose split fails are queued by their A lane for
   fdgpu_full_kernel exactly as the one-lane kernel queues them (the A
   table, the parked R, k's digits and [S]B are in the signature's own
   workspace). */

/* [|d|](+-T) for one table, digits pre-shifted so that digit nwin-1 sits in
   the top nibble; staged through LDS like hs_chain (one entry per window). */
FDG_DEV void hs_chain1(ge_p1p1 &t, uint32_t (&dd)[5], bool neg, uint32_t nwin, const uint32_t *tab) {
  __shared__ uint32_t s_stage1[FDGPU_BLOCK / 64][10 * 256];
  uint32_t *st = &s_stage1[threadIdx.x >> 6][0];
  ge_p2 acc2;
  ge_p3 acc3;
  uint32_t q[40];
  {                                             /* top window: O + T[d] */
    const int d = sext4(dd[4] >> 28);
    shl4_5(dd);
    atab_load(q, tab, d);
    ge_p3_0(acc3);
    ge_add_cached_regs(t, acc3, q, (d < 0) != neg);
  }
#pragma unroll 1
  for (uint32_t j = 1; j < nwin; j++) {
    ge_p1p1_to_p2(acc2, t);
    const int d = sext4(dd[4] >> 28);
    shl4_5(dd);
    stage_entry(st, tab, d);
#pragma unroll 1
    for (int r = 0; r < 4; r++) {
      ge_dbl(t, acc2);
      ge_p1p1_to_p2(acc2, t);
    }
    acc3.X = acc2.X; acc3.Y = acc2.Y; acc3.Z = acc2.Z; fe_mul(acc3.T, t.X, t.Y);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   /* the window's LDS-DMA has landed */
    unstage_entry_signed(q, st, (d < 0) != neg);
    ge_add_cached_regs_swapped(t, acc3, q, (d < 0) != neg);
  }
}

FDG_DEV void fe_xchg_pair(fe &r, const fe &a) {
#pragma unroll
  for (int j = 0; j < 10; j++) r.v[j] = (uint32_t)__shfl_xor((int)a.v[j], 1);
}

__global__ void __launch_bounds__(FDGPU_BLOCK, FDGPU_VERIFY_WAVES)
fdgpu_verify_pair_kernel(const uint8_t *__restrict__ arena, const fdgpu_sig_desc_t *__restrict__ sigs, uint32_t n_sig_arg,
                         const uint32_t *__restrict__ n_sig_dev, const uint32_t *__restrict__ btab,
                         uint32_t *__restrict__ ws, const uint32_t *__restrict__ perm, int8_t *__restrict__ codes,
                         uint32_t *__restrict__ queue, uint32_t *__restrict__ queue_cnt, uint32_t flags) {
  const uint32_t n_sig = n_sig_dev ? *n_sig_dev : n_sig_arg;
  if (blockIdx.x * (blockDim.x / 2u) >= n_sig) return;
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x, i = g >> 1;
  const bool rl = (g & 1u) != 0;                /* the R lane of signature i (else its A lane) */
  const bool active = i < n_sig;
  const bool ref_map = (flags & FDGPU_FLAG_REF_MAP) != 0;
  const fdgpu_sig_desc_t d = sigs[active ? i : n_sig - 1];
  uint32_t nb = sha512_hram_blocks(d.msg_sz);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) nb = max(nb, (uint32_t)__shfl_xor((int)nb, off));
  uint32_t *wsl = lane_ws(ws, i);             /* i < the workspace's lanes: ceil(n / 128) x 128 <= ceil(n / 256) x 256 */
  uint32_t *park = wsl + FDGPU_WS_PARK * FDGPU_ATAB_WORDS;
  uint32_t Renc[8], Aenc[8];
  load32(Renc, arena + d.sig_off);
  load32(Aenc, arena + d.pub_off);
  uint32_t k[8];
  {
    uint64_t h[8];
    sha512_hram(h, Renc, Aenc, arena + d.msg_off, d.msg_sz, nb);
    uint32_t kx[16];
#pragma unroll
    for (int j = 0; j < 8; j++) { kx[2 * j] = bswap32((uint32_t)(h[j] >> 32)); kx[2 * j + 1] = bswap32((uint32_t)h[j]); }
    sc_reduce512(k, kx);
  }
  uint32_t S[8];
  load32(S, arena + d.sig_off + 32);
  int code = sc_lt_L(S) ? 0 : -1;
#pragma unroll
  for (int j = 0; j < 8; j++) S[j] = code ? 0u : S[j];
  /* each lane decodes its own point and builds its table */
  {
    uint32_t enc[8];
#pragma unroll
    for (int j = 0; j < 8; j++) enc[j] = rl ? Renc[j] : Aenc[j];
    ge_p3 P, Pn;
    const bool ok = ge_decode(P, enc, ref_map);
    const bool small = ge_is_small_order_affine(P);
    ge_p3_neg(Pn, P);
    atab_build(rl ? tab_r(wsl) : tab_a(wsl), Pn);
    /* both verdicts in both lanes, in decode2's order (A first) */
    const uint32_t mine = (ok ? 1u : 0u) | (small ? 2u : 0u);
    const uint32_t other = (uint32_t)__shfl_xor((int)mine, 1);
    const uint32_t av = rl ? other : mine, rv = rl ? mine : other;
    if (code == 0 && !(av & 1u)) code = ref_map ? -2 : -1;
    if (code == 0 && !(rv & 1u)) code = -1;
    if (code == 0 && (av & 2u)) code = -2;                 /* fd_ed25519_user.c:194-199 */
    if (code == 0 && (rv & 2u)) code = -1;
  }
  const bool need = active && code == 0;
  hs_split_t hs;
  {
    uint32_t ke[8];
#pragma unroll
    for (int j = 0; j < 8; j++) ke[j] = need ? k[j] : 0u;
    hs_split(hs, ke);
  }
  uint32_t ud[5], vd[5], ndu = 0, ndv = 0;
  recode16_160(ud, ndu, hs.u);
  recode16_160(vd, ndv, hs.v);
  const uint32_t nd_lane = max(max(ndu, ndv), 1u);
  const bool full = need && (!hs.ok || nd_lane > HS_MAX_WIN || (flags & FDGPU_FLAG_KFULL));
  const bool half = need && !full;
  {
    uint32_t w[8];
    hs_wscalar(w, hs.v, hs.v_neg, S);
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = half ? w[j] : S[j];
    /* the A lane sums the comb's low tables, the R lane its high ones; the
       halves are exchanged and added */
    ge_p3 WB, WBo;
    comb_sb(WB, w, btab, rl ? BC_NDIG / 2u : 0u, rl ? BC_NDIG : BC_NDIG / 2u);
    fe_xchg_pair(WBo.X, WB.X);
    fe_xchg_pair(WBo.Y, WB.Y);
    fe_xchg_pair(WBo.Z, WB.Z);
    fe_xchg_pair(WBo.T, WB.T);
    ge_cached c; ge_p3_to_cached(c, WBo);
    ge_p1p1 tw; ge_add_cached(tw, WB, c, false);
    ge_p1p1_to_p3(WB, tw);
    ge_p3_to_cached(c, WB);
    if (!rl) atab_store(wsl, FDGPU_WS_SB, c);
  }
  if (full && !rl) {
    uint32_t kd[KD_WORDS];
    sc_recode16(kd, k);
#pragma unroll
    for (int j = 0; j < KD_WORDS; j++) park[HPARK_KD + j] = kd[j];
    park[HPARK_CODE] = 0u;
  }
  bool eq = false;
  if (__any(half)) {
    uint32_t nwin = half ? nd_lane : 1u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nwin = max(nwin, (uint32_t)__shfl_xor((int)nwin, off));
    uint32_t dd[5];
#pragma unroll
    for (int j = 0; j < 5; j++) dd[j] = rl ? vd[j] : ud[j];
#pragma unroll 1
    for (uint32_t s2 = nwin; s2 < 40; s2++) shl4_5(dd);
    ge_p1p1 t;
    hs_chain1(t, dd, rl ? hs.v_neg : hs.u_neg, nwin, rl ? tab_r(wsl) : tab_a(wsl));
    /* exchange the halves and add: both lanes hold [u](-A) + [v](-R) */
    ge_p3 mine, other;
    ge_p1p1_to_p3(mine, t);
    fe_xchg_pair(other.X, mine.X);
    fe_xchg_pair(other.Y, mine.Y);
    fe_xchg_pair(other.Z, mine.Z);
    fe_xchg_pair(other.T, mine.T);
    ge_cached oc;
    ge_p3_to_cached(oc, other);
    ge_add_cached(t, mine, oc, false);
    /* chain == -[w]B (the A lane parked [w]B; a lane reads its own pair's entry) */
    uint32_t q[40];
    atab_load(q, wsl, (int)FDGPU_WS_SB);
    fe ypx, ymx, z2, xw, yw, l1, l2;
#pragma unroll
    for (int j = 0; j < 10; j++) { ypx.v[j] = q[j]; ymx.v[j] = q[10 + j]; z2.v[j] = q[20 + j]; }
    fe_sub(xw, ypx, ymx);
    fe_add(yw, ypx, ymx);
    fe_mul(l1, t.X, z2);
    fe_mul(l2, t.Z, xw);
    fe_add(l1, l1, l2);
    const bool ex = fe_iszero(l1);
    fe_mul(l1, t.Y, z2);
    fe_mul(l2, t.T, yw);
    fe_sub(l1, l1, l2);
    eq = ex && fe_iszero(l1);
  }
  if (active && !full && !rl) codes[out_idx(perm, i)] = (int8_t)(code ? code : (eq ? 0 : -3));
  {
    const bool q_full = full && !rl;
    const uint64_t m = __ballot(q_full);
    if (m) {
      const int lane = (int)(threadIdx.x & 63u);
      const int leader = __ffsll((long long)m) - 1;
      uint32_t base = 0;
      if (lane == leader) base = atomicAdd(queue_cnt, (uint32_t)__popcll(m));
      base = (uint32_t)__shfl((int)base, leader, 64);
      if (q_full) queue[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = i;
    }
  }
}

/* ---------------- key cache (FDGPU_FLAG_KCACHE) ----------------
   Signers repeat within a batch (a vote account signs every slot).  Each
   distinct public key is decoded and its -A table built once, in the
   workspace of one representative lane; the verify and fallback kernels'
   other lanes with that key read that table in place instead of
   decompressing A (a 2^252-3 exponentiation) and building their own.
   Results are unchanged: the decode is a function of the 32 key bytes only.

   fdgpu_key_dedup_kernel: an open-addressing table of signature indices,
   keyed by a seeded hash of all 32 key bytes.  A lane claims an empty slot
   with atomicCAS (after a plain load saw it empty), or compares its key with
   the bytes of the index a slot already holds (the arena is immutable, so
   nothing waits on another lane).  After KC_PROBES probes it stays its own
   representative, which bounds the work whatever keys a batch carries.  key_of[i] = representative of i;
   the representatives are appended to reps (compact, so the table kernel
   runs dense waves however they are scattered over the batch). */
#define KC_PROBES 32u
#define KC_EMPTY 0xffffffffu

FDG_DEV uint32_t kc_hash(const uint32_t (&a)[8], uint64_t seed) {
  uint64_t h = seed;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    h ^= ((uint64_t)a[2 * j + 1] << 32) | a[2 * j];
    h *= 0x9e3779b97f4a7c15ull;
    h ^= h >> 29;
  }
  h *= 0xbf58476d1ce4e5b9ull;
  return (uint32_t)(h >> 32) ^ (uint32_t)h;
}

__global__ void __launch_bounds__(256) fdgpu_key_dedup_kernel(const uint8_t *__restrict__ arena,
                                                              const fdgpu_sig_desc_t *__restrict__ sigs,
                                                              uint32_t n_sig_arg, const uint32_t *__restrict__ n_sig_dev,
                                                              uint32_t *__restrict__ ht, uint32_t ht_mask,
                                                              uint32_t *__restrict__ key_of, uint32_t *__restrict__ reps,
                                                              uint32_t *__restrict__ rep_cnt, uint64_t seed) {
  const uint32_t n_sig = n_sig_dev ? *n_sig_dev : n_sig_arg;
  if (blockIdx.x * blockDim.x >= n_sig) return;     /* whole block: the barriers below need every thread */
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  bool is_rep = false;
  if (i < n_sig) {
    uint32_t a[8];
    load32(a, arena + sigs[i].pub_off);
    uint32_t slot = kc_hash(a, seed) & ht_mask, rep = i;
    for (uint32_t p = 0; p < KC_PROBES; p++, slot = (slot + 1u) & ht_mask) {
      /* a plain load first: a signer's slot is taken by its first signature,
         and the many later ones then compare without an atomic on a hot line */
      uint32_t v = ht[slot];                        /* stale only as EMPTY: the CAS then reads it */
      if (v == KC_EMPTY) {
        v = atomicCAS(&ht[slot], KC_EMPTY, i);
        if (v == KC_EMPTY) break;                   /* claimed: i represents its key */
      }
      uint32_t b[8];
      load32(b, arena + sigs[v].pub_off);
      uint32_t diff = 0;
#pragma unroll
      for (int j = 0; j < 8; j++) diff |= a[j] ^ b[j];
      if (!diff) { rep = v; break; }
    }
    key_of[i] = rep;
    is_rep = rep == i;
  }
  /* append the representatives: wave offsets in LDS, one global atomic per
     workgroup (a single counter takes every one of them) */
  __shared__ uint32_t s_cnt, s_base;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const uint64_t m = __ballot(is_rep);
  const int lane = (int)(threadIdx.x & 63u);
  uint32_t wbase = 0;
  if (m && lane == __ffsll((long long)m) - 1) wbase = atomicAdd(&s_cnt, (uint32_t)__popcll(m));
  if (m) wbase = (uint32_t)__shfl((int)wbase, __ffsll((long long)m) - 1, 64);
  __syncthreads();
  if (threadIdx.x == 0) s_base = s_cnt ? atomicAdd(rep_cnt, s_cnt) : 0u;
  __syncthreads();
  if (is_rep) reps[s_base + wbase + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = i;
}

/* One lane per representative: decode A, small-order test, -A table into the
   representative's own workspace, verdict (bit 0 decoded, bit 1 small
   order) into kverd.  The grid covers every signature; blocks past the
   representative count leave at once. */
__global__ void __launch_bounds__(FDGPU_BLOCK, FDGPU_VERIFY_WAVES)
fdgpu_key_table_kernel(const uint8_t *__restrict__ arena, const fdgpu_sig_desc_t *__restrict__ sigs,
                       uint32_t *__restrict__ ws, const uint32_t *__restrict__ reps,
                       const uint32_t *__restrict__ rep_cnt, uint32_t *__restrict__ kverd, uint32_t flags) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= *rep_cnt) return;
  const uint32_t i = reps[q];
  uint32_t Aenc[8];
  load32(Aenc, arena + sigs[i].pub_off);
  ge_p3 P, Pn;
  const bool a_ok = ge_decode(P, Aenc, (flags & FDGPU_FLAG_REF_MAP) != 0);
  const bool a_small = ge_is_small_order_affine(P);
  ge_p3_neg(Pn, P);
  atab_build(tab_a(lane_ws(ws, i)), Pn);
  kverd[i] = (a_ok ? 1u : 0u) | (a_small ? 2u : 0u);
}

/* The queued lanes of fdgpu_verify_hs_kernel: [S]B + [k](-A) with k's 64
   windows (dsm_k), compared with the decoded R (from the lane's -R table). */
__global__ void __launch_bounds__(FDGPU_BLOCK, FDGPU_VERIFY_WAVES)
fdgpu_full_kernel(uint32_t *__restrict__ ws, const uint32_t *__restrict__ perm, int8_t *__restrict__ codes,
                  const uint32_t *__restrict__ queue, const uint32_t *__restrict__ queue_cnt, uint32_t slots,
                  const uint32_t *__restrict__ key_of);

FDG_DEV void full_body(uint32_t *__restrict__ ws, const uint32_t *__restrict__ perm, int8_t *__restrict__ codes,
                       const uint32_t *__restrict__ queue, const uint32_t *__restrict__ queue_cnt, uint32_t slots,
                       const uint32_t *__restrict__ key_of, uint32_t bx) {
  const uint32_t cnt = *queue_cnt;
  if (bx * blockDim.x >= cnt) return;
  for (uint32_t q = bx * blockDim.x + threadIdx.x; q < cnt; q += slots) {
    const uint32_t i = queue[q];
    uint32_t *wsl = ws + (size_t)i * FDGPU_WS_LANE_WORDS;
    const uint32_t *park = wsl + FDGPU_WS_PARK * FDGPU_ATAB_WORDS;
    uint32_t kd[KD_WORDS];
#pragma unroll
    for (int j = 0; j < KD_WORDS; j++) kd[j] = park[HPARK_KD + j];
    ge_p2 Rc;
    dsm_k(Rc, kd, wsl, FDGPU_WS_SB, tab_a(key_of ? lane_ws(ws, key_of[i]) : wsl));
    /* == R: the -R table's entry 1 is (Y-X, Y+X, 2Z, -2dT) of R = (X:Y:Z),
       so 2X = YmX - YpX and 2Y = YpX + YmX; compare X / Z, Y / Z crosswise */
    uint32_t er[40];
    atab_load(er, tab_r(wsl), 1);
    fe ypx, ymx, z2, x2, y2, l, r;
#pragma unroll
    for (int j = 0; j < 10; j++) { ypx.v[j] = er[j]; ymx.v[j] = er[10 + j]; z2.v[j] = er[20 + j]; }
    fe_carry(ypx); fe_carry(ymx); fe_carry(z2);
    fe_sub(x2, ymx, ypx);
    fe_add(y2, ypx, ymx);
    fe_mul(l, Rc.X, z2); fe_mul(r, x2, Rc.Z);
    bool eq = fe_eq(l, r);
    fe_mul(l, Rc.Y, z2); fe_mul(r, y2, Rc.Z);
    eq = eq && fe_eq(l, r);
    codes[out_idx(perm, i)] = (int8_t)(eq ? 0 : -3);
  }
}

__global__ void __launch_bounds__(FDGPU_BLOCK, FDGPU_VERIFY_WAVES)
fdgpu_full_kernel(uint32_t *__restrict__ ws, const uint32_t *__restrict__ perm, int8_t *__restrict__ codes,
                  const uint32_t *__restrict__ queue, const uint32_t *__restrict__ queue_cnt, uint32_t slots,
                  const uint32_t *__restrict__ key_of) {
  full_body(ws, perm, codes, queue, queue_cnt, slots, key_of, blockIdx.x);
}

/* the fallback of a merged verify: block (x, y) serves batch y's queue */
__global__ void __launch_bounds__(FDGPU_BLOCK, FDGPU_VERIFY_WAVES)
fdgpu_full_multi_kernel(const fdgpu_mbatch_t *__restrict__ mb) {
  const fdgpu_mbatch_t b = mb[blockIdx.y];
  if (blockIdx.x >= b.slow) return;
  full_body(b.ws, nullptr, b.codes, b.queue, b.cnt, b.slow * FDGPU_BLOCK, nullptr, blockIdx.x);
}

/* Per transaction: fd_ed25519_verify_batch_single_msg's first-error order
   (fd_ed25519_user.c:232-310) over its signatures' codes, plus the batch's
   accept/reject results compacted by wavefront ballot: bit t of accept[]
   is set iff transaction t verified (one 64-bit word per wave; the verify
   tile only needs accept/reject, so it can read n/8 bytes instead of n). */
__global__ void __launch_bounds__(256) fdgpu_combine_kernel(const fdgpu_txn_desc_t *__restrict__ txns, uint32_t n_txn,
                                                            const int8_t *__restrict__ sig_codes,
                                                            int8_t *__restrict__ txn_codes,
                                                            uint64_t *__restrict__ accept) {
  /* FDGPU_AUX_BLOCKS blocks stride over the batch, 256 txns a step */
  for (uint32_t t0 = blockIdx.x * blockDim.x; t0 < n_txn; t0 += gridDim.x * blockDim.x) {
    const uint32_t t = t0 + threadIdx.x;
    int code = -1;
    if (t < n_txn) {
      const fdgpu_txn_desc_t d = txns[t];
      if (d.sig_cnt >= 1 && d.sig_cnt <= 16) {             /* else ERR_SIG (fd_ed25519_user.c:238-241) */
        int first_struct = 0, any_msg = 0;
        for (uint32_t j = 0; j < d.sig_cnt; j++) {
          const int c = sig_codes[d.sig0 + j];
          if (c == -3) any_msg = 1;
          else if (c != 0 && first_struct == 0) first_struct = c;
        }
        /* pass 1 reports its first failure before any pass-2 (equation) failure */
        code = first_struct ? first_struct : (any_msg ? -3 : 0);
      }
      txn_codes[t] = (int8_t)code;
    }
    const uint64_t ok = __ballot(t < n_txn && code == 0);   /* every lane of the wave takes part */
    if (accept && (threadIdx.x & 63u) == 0 && t < n_txn) accept[t >> 6] = ok;
  }
}

/* ---------------- test / diagnostic kernels ---------------- */

/* in: n records of 2 x 8 u32 (a, b < 2^255 as LE words); out: n records of
   8 ops x 8 u32 canonical: a*b, a^2, a+b, a-b, pow22523(a), invert(a), canon(a), -a */
__global__ void __launch_bounds__(64) fdgpu_test_fe_kernel(const uint32_t *in, uint32_t *out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t aw[8], bw[8];
#pragma unroll
  for (int j = 0; j < 8; j++) { aw[j] = in[16 * i + j]; bw[j] = in[16 * i + 8 + j]; }
  fe a, b, r;
  fe_frombytes(a, aw); fe_frombytes(b, bw);
  uint32_t o[8];
  uint32_t *dst = out + 64 * i;
  fe_mul(r, a, b); fe_tobytes(o, r);
  for (int j = 0; j < 8; j++) dst[j] = o[j];
  fe_sq(r, a); fe_tobytes(o, r);
  for (int j = 0; j < 8; j++) dst[8 + j] = o[j];
  fe_add(r, a, b); fe_tobytes(o, r);
  for (int j = 0; j < 8; j++) dst[16 + j] = o[j];
  fe_sub(r, a, b); fe_tobytes(o, r);
  for (int j = 0; j < 8; j++) dst[24 + j] = o[j];
  fe_pow22523(r, a); fe_tobytes(o, r);
  for (int j = 0; j < 8; j++) dst[32 + j] = o[j];
  fe_invert(r, a); fe_tobytes(o, r);
  for (int j = 0; j < 8; j++) dst[40 + j] = o[j];
  fe_tobytes(o, a);
  for (int j = 0; j < 8; j++) dst[48 + j] = o[j];
  fe_neg(r, a); fe_tobytes(o, r);
  for (int j = 0; j < 8; j++) dst[56 + j] = o[j];
}

/* in: n encodings (8 u32); out: n x 18 u32: [rc, small_order, x(8), y(8)] */
__global__ void __launch_bounds__(64) fdgpu_test_decode_kernel(const uint32_t *enc, uint32_t *out, uint32_t n, uint32_t flags) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t e[8];
  for (int j = 0; j < 8; j++) e[j] = enc[8 * i + j];
  ge_p3 P;
  const bool ok = ge_decode(P, e, (flags & FDGPU_FLAG_REF_MAP) != 0);
  uint32_t *dst = out + 18 * i;
  dst[0] = ok ? 0u : 0xffffffffu;
  dst[1] = ok ? (ge_is_small_order_affine(P) ? 1u : 0u) : 0xffffffffu;
  uint32_t x[8], y[8];
  fe_tobytes(x, P.X); fe_tobytes(y, P.Y);
  for (int j = 0; j < 8; j++) { dst[2 + j] = x[j]; dst[10 + j] = y[j]; }
}

/* SHA-512 of arena[msg_off .. +msg_sz]; out: n x 16 u32 (digest bytes, LE words) */
__global__ void __launch_bounds__(64) fdgpu_test_sha512_kernel(const uint8_t *arena, const fdgpu_sig_desc_t *msgs, uint32_t n,
                                         uint32_t *out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = i < n;
  const fdgpu_sig_desc_t d = msgs[active ? i : n - 1];
  uint32_t nb = (d.msg_sz + 16u) / 128u + 1u;
  for (int off = 32; off > 0; off >>= 1) nb = max(nb, (uint32_t)__shfl_xor((int)nb, off));
  uint64_t h[8];
  sha512_plain(h, arena + d.msg_off, d.msg_sz, nb);
  if (!active) return;
  for (int j = 0; j < 8; j++) {
    out[16 * i + 2 * j] = bswap32((uint32_t)(h[j] >> 32));
    out[16 * i + 2 * j + 1] = bswap32((uint32_t)h[j]);
  }
}

/* k = SHA-512(R||A||M) mod L per signature; out: n x 8 u32 */
__global__ void __launch_bounds__(64) fdgpu_test_hram_kernel(const uint8_t *arena, const fdgpu_sig_desc_t *sigs, uint32_t n,
                                       uint32_t *out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = i < n;
  const fdgpu_sig_desc_t d = sigs[active ? i : n - 1];
  uint32_t nb = sha512_hram_blocks(d.msg_sz);
  for (int off = 32; off > 0; off >>= 1) nb = max(nb, (uint32_t)__shfl_xor((int)nb, off));
  uint32_t R[8], A[8];
  load32(R, arena + d.sig_off);
  load32(A, arena + d.pub_off);
  uint64_t h[8];
  sha512_hram(h, R, A, arena + d.msg_off, d.msg_sz, nb);
  uint32_t kx[16], k[8];
  for (int j = 0; j < 8; j++) { kx[2 * j] = bswap32((uint32_t)(h[j] >> 32)); kx[2 * j + 1] = bswap32((uint32_t)h[j]); }
  sc_reduce512(k, kx);
  if (!active) return;
  for (int j = 0; j < 8; j++) out[8 * i + j] = k[j];
}

__global__ void __launch_bounds__(64) fdgpu_test_sc_reduce_kernel(const uint32_t *in, uint32_t *out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x[16], r[8];
  for (int j = 0; j < 16; j++) x[j] = in[16 * i + j];
  sc_reduce512(r, x);
  for (int j = 0; j < 8; j++) out[8 * i + j] = r[j];
}

/* ---------------- GPU-side ingest ----------------
   Raw transaction payloads -> the verify's descriptors, on the device:
     parse   one payload per lane through fdt_parse_core (fdt_parse.h, the
             host parser's own source): the fd_txn_t (which the verify tile
             writes into its output trailer), its footprint (0: not a
             transaction), and the signature layout -- signatures at
             signature_off, the signer keys are the first sig_cnt account
             addresses, the message runs from message_off to the end;
     scan    exclusive prefix sum of the per-txn signature counts (a count
             outside [1,16] contributes none: batch_single_msg rejects the
             txn unverified, fd_ed25519_user.c:238-241) -> each txn's first
             signature and the batch's signature count, left on the device;
     expand  the per-signature descriptors, in transaction order.
   A valid txn with s signatures is at least 96 s + 38 bytes (s signatures,
   s signer keys, blockhash, the counts), which bounds the signature count
   of a batch from its frag sizes alone (fdgpu_frag_sig_bound). */
#define FDGPU_SCAN_BLOCK 1024u      /* txns per scan block: 256 threads x 4 */


/* frag t's {off, sz} are the first two words of a record of `stride` words
   (fdgpu_frag_t: 2, fdgpu_frag_ex_t: 4) */
__global__ void __launch_bounds__(64) fdgpu_frag_parse_kernel(
    const uint8_t *__restrict__ arena, const uint32_t *__restrict__ frags, uint32_t stride, uint32_t n,
    uint8_t *__restrict__ txn_out, uint16_t *__restrict__ txn_sz, fdgpu_txn_t *__restrict__ txd,
    uint32_t *__restrict__ cnt) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const fdgpu_frag_t f = *(const fdgpu_frag_t *)(frags + (size_t)t * stride);
  fdt_txn_t *x = (fdt_txn_t *)(txn_out + (size_t)t * FDT_TXN_MAX_SZ);
  uint64_t why = 0;
  uint64_t fp = fdt_parse_core(arena + f.off, f.sz, x, &why);
  const uint32_t sc = fp ? x->signature_cnt : 0u;
  uint32_t c = (sc >= 1u && sc <= 16u) ? sc : 0u;
  if (c > fdt_frag_sig_bound(f.sz)) { c = 0u; fp = 0u; }       /* cannot happen for a parsed txn (see above) */
  fdgpu_txn_t d;
  d.msg_off = fp ? f.off + x->message_off : f.off;
  d.msg_sz = fp ? f.sz - x->message_off : 0u;
  d.sig_off = fp ? f.off + x->signature_off : f.off;
  d.pub_off = fp ? f.off + x->acct_addr_off : f.off;
  d.sig_cnt = fp ? sc : 0u;
  txd[t] = d;
  cnt[t] = c;
  txn_sz[t] = (uint16_t)fp;
}

/* Inclusive scan of v over the 64 lanes of a wave */
FDG_DEV uint32_t wave_incl_scan(uint32_t v) {
  const int lane = (int)(threadIdx.x & 63u);
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t u = (uint32_t)__shfl_up((int)v, off, 64);
    v += lane >= off ? u : 0u;
  }
  return v;
}

/* Block-local exclusive scan of cnt over FDGPU_SCAN_BLOCK txns -> sig0
   (local), the block's total -> blocktot */
__global__ void __launch_bounds__(256) fdgpu_scan_local_kernel(const uint32_t *__restrict__ cnt, uint32_t n,
                                                               uint32_t *__restrict__ sig0,
                                                               uint32_t *__restrict__ blocktot) {
  __shared__ uint32_t s_wave[4];
  const uint32_t base = blockIdx.x * FDGPU_SCAN_BLOCK + threadIdx.x * 4u;
  uint32_t v[4], sum = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) { v[k] = base + k < n ? cnt[base + k] : 0u; sum += v[k]; }
  const uint32_t incl = wave_incl_scan(sum);
  const uint32_t wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63u) == 63u) s_wave[wv] = incl;
  __syncthreads();
  uint32_t off = incl - sum;
  for (uint32_t w = 0; w < wv; w++) off += s_wave[w];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (base + k < n) sig0[base + k] = off;
    off += v[k];
  }
  if (threadIdx.x == 255u) blocktot[blockIdx.x] = off;
}

/* One block: exclusive scan of the nb block totals (in place) and the
   grand total -> *n_sig */
__global__ void __launch_bounds__(1024) fdgpu_scan_blocks_kernel(uint32_t *__restrict__ blocktot, uint32_t nb,
                                                                 uint32_t *__restrict__ n_sig) {
  __shared__ uint32_t s_wave[16];
  __shared__ uint32_t s_carry;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  for (uint32_t b0 = 0; b0 < nb; b0 += 1024u) {
    const uint32_t i = b0 + threadIdx.x;
    const uint32_t v = i < nb ? blocktot[i] : 0u;
    const uint32_t incl = wave_incl_scan(v);
    const uint32_t wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 63u) s_wave[wv] = incl;
    __syncthreads();
    uint32_t off = s_carry + incl - v;
    for (uint32_t w = 0; w < wv; w++) off += s_wave[w];
    __syncthreads();
    if (i < nb) blocktot[i] = off;
    if (threadIdx.x == 1023u) s_carry = off + v;
    __syncthreads();
  }
  if (threadIdx.x == 0) *n_sig = s_carry;
}

/* One thread per txn: its combine item and its signatures' descriptors */
__global__ void __launch_bounds__(256) fdgpu_frag_expand_kernel(
    const fdgpu_txn_t *__restrict__ txd, const uint32_t *__restrict__ cnt, const uint32_t *__restrict__ sig0,
    const uint32_t *__restrict__ blockoff, uint32_t n, fdgpu_sig_desc_t *__restrict__ sigs,
    fdgpu_txn_desc_t *__restrict__ tds) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint32_t c = cnt[t], s0 = sig0[t] + blockoff[t / FDGPU_SCAN_BLOCK];
  fdgpu_txn_desc_t td;
  td.sig0 = s0;
  td.sig_cnt = c;
  tds[t] = td;
  if (!c) return;
  const fdgpu_txn_t d = txd[t];
  for (uint32_t j = 0; j < c; j++) {
    fdgpu_sig_desc_t sd;
    sd.msg_off = d.msg_off;
    sd.msg_sz = d.msg_sz;
    sd.sig_off = d.sig_off + 64u * j;
    sd.pub_off = d.pub_off + 32u * j;
    sigs[s0 + j] = sd;
  }
}

/* Ring-slot frag batches of up to FDGPU_SMALL_SCAN_MAX txns: the
   signature-count scan and the descriptor expansion in ONE block (1024
   threads, each a run of consecutive txns), instead of the three-kernel
   multi-block scan: a verify tile's batch costs two launches fewer. */
__global__ void __launch_bounds__(1024) fdgpu_frag_scan_expand_small_kernel(
    const fdgpu_txn_t *__restrict__ txd, const uint32_t *__restrict__ cnt, uint32_t n,
    fdgpu_sig_desc_t *__restrict__ sigs, fdgpu_txn_desc_t *__restrict__ tds, uint32_t *__restrict__ n_sig) {
  __shared__ uint32_t s_wave[16];
  const uint32_t per = (n + 1023u) / 1024u, t0 = threadIdx.x * per, t1 = min(n, t0 + per);
  uint32_t sum = 0;
  for (uint32_t t = t0; t < t1; t++) sum += cnt[t];
  const uint32_t incl = wave_incl_scan(sum);
  const uint32_t wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63u) == 63u) s_wave[wv] = incl;
  __syncthreads();
  uint32_t off = incl - sum;
  for (uint32_t w = 0; w < wv; w++) off += s_wave[w];
  if (threadIdx.x == 1023u) *n_sig = off + sum;
  for (uint32_t t = t0; t < t1; t++) {
    const uint32_t c = cnt[t];
    fdgpu_txn_desc_t td;
    td.sig0 = off;
    td.sig_cnt = c;
    tds[t] = td;
    if (c) {
      const fdgpu_txn_t d = txd[t];
      for (uint32_t j = 0; j < c; j++) {
        fdgpu_sig_desc_t sd;
        sd.msg_off = d.msg_off;
        sd.msg_sz = d.msg_sz;
        sd.sig_off = d.sig_off + 64u * j;
        sd.pub_off = d.pub_off + 32u * j;
        sigs[off + j] = sd;
      }
    }
    off += c;
  }
}

/* The end of a ring-slot frag batch in one launch, per txn: the
   batch_single_msg combine of its signatures' codes, FDGPU_CODE_PARSE_FAIL
   for a payload that is not a transaction, and its parsed fd_txn_t copied
   to the place the caller reserved (from the payload's counts,
   fdt_txn_peek) -- a footprint other than the reservation (only a caller
   bug can cause one) gets FDGPU_CODE_TRAILER_CAP and no verdict.  codes and
   trailers are one buffer (trailers after the codes), copied back in one
   transfer.  Lane per txn; tr_off is 4-byte aligned, the txn record starts
   a 852-B (4-aligned) stride. */
__global__ void __launch_bounds__(256) fdgpu_frag_finish_kernel(const fdgpu_txn_desc_t *__restrict__ txns, uint32_t n,
                                                                const int8_t *__restrict__ sig_codes,
                                                                const uint16_t *__restrict__ txn_sz,
                                                                const fdgpu_frag_ex_t *__restrict__ fx,
                                                                const uint8_t *__restrict__ txn_out,
                                                                int8_t *__restrict__ codes, uint8_t *__restrict__ trailers) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint32_t fp = txn_sz[t];
  int code = -1;
  if (!fp) {
    code = FDGPU_CODE_PARSE_FAIL;
  } else {
    const fdgpu_frag_ex_t f = fx[t];
    if (fp != f.tr_cap) {
      code = FDGPU_CODE_TRAILER_CAP;
    } else {
      const fdgpu_txn_desc_t d = txns[t];
      if (d.sig_cnt >= 1 && d.sig_cnt <= 16) {           /* else ERR_SIG (fd_ed25519_user.c:238-241) */
        int first_struct = 0, any_msg = 0;
        for (uint32_t j = 0; j < d.sig_cnt; j++) {
          const int c = sig_codes[d.sig0 + j];
          if (c == -3) any_msg = 1;
          else if (c != 0 && first_struct == 0) first_struct = c;
        }
        code = first_struct ? first_struct : (any_msg ? -3 : 0);
      }
      const uint32_t *src = (const uint32_t *)(txn_out + (size_t)t * FDT_TXN_MAX_SZ);
      uint32_t *dst = (uint32_t *)(trailers + f.tr_off);
      for (uint32_t w = 0; w < (fp + 3u) / 4u; w++) dst[w] = src[w];
    }
  }
  codes[t] = (int8_t)code;
}

/* Gathered frag batches (fdgpu_submit_frags_io).  Both kernels run on at
   most FDGPU_IO_BLOCKS blocks (fdgpu_internal.h: a workgroup beside the
   verify holds a verify block's slot while it waits on the bus) and each wave
   strides over groups of 64 frags, lane i of a group owning frag 64 g + i. */

/* the group's lane that owns flattened unit k: the first lane whose
   inclusive unit count exceeds k (incl is non-decreasing over the lanes) */
FDG_DEV uint32_t unit_owner(uint32_t incl, uint32_t k) {
  uint32_t o = 0;
#pragma unroll
  for (uint32_t b = 32; b; b >>= 1)
    if ((uint32_t)__shfl((int)incl, (int)(o + b - 1u), 64) <= k) o += b;
  return o;
}

/* Ingest: per group, lane i reads frag i's record and payload address from
   the slot's pinned upload buffer (one coalesced read of each over the bus),
   then the wave copies the group's payloads from host memory (the registered
   in dcache, read in place) to their packed, 16-B aligned places in the batch
   arena -- the payloads' 16-B units flattened over the group, four loads in
   flight per lane (the units past sz lie in the payload's own 64-B chunks).
   With chk, a frag whose pair {line, seq} names an in-mcache line is then
   re-checked as the reference's mux re-checks after its copy (fd_mux.c:
   641-655): once the wave's payload loads have returned, the line's seq is
   read again over the bus (a system-scope load: no cache in between); any
   other value than the frag's seq means the producer republished the line,
   so its payload may have been rewritten under the read, and the record is
   kept with FDGPU_FX_LAPPED set (no parse, no verdict).  An agent-scope
   acquire (L1 invalidate) then makes the copied bytes visible to the
   group's own loads, and lane i parses frag i (fd_txn_parse,
   fdgpu_frag_parse_kernel's parse) and the wave takes its run of descriptor
   slots with one atomic add on *n_sig, so the descriptors stay dense in
   [0, n_sig) grouped by wave (every txn records its own first slot).  The
   records are kept on the device (fx_dev) for the finish kernel; the first
   thread clears the verify kernel's queue counter (zero_word). */
__global__ void __launch_bounds__(256) fdgpu_frag_ingest_io_kernel(
    const uint64_t *__restrict__ src, const fdgpu_frag_ex_t *__restrict__ fx, const uint64_t *__restrict__ chk,
    const uint64_t *__restrict__ rtab, uint32_t n, uint8_t *__restrict__ arena, fdgpu_frag_ex_t *__restrict__ fx_dev,
    uint8_t *__restrict__ txn_out, uint16_t *__restrict__ txn_sz, fdgpu_sig_desc_t *__restrict__ sigs,
    fdgpu_txn_desc_t *__restrict__ tds, uint32_t *__restrict__ n_sig, uint32_t *__restrict__ zero_word) {
  const uint32_t lane = threadIdx.x & 63u, wpb = blockDim.x >> 6;
  if (blockIdx.x == 0 && threadIdx.x == 0 && zero_word) *zero_word = 0u;
  for (uint32_t g = blockIdx.x * wpb + (threadIdx.x >> 6); g * 64u < n; g += gridDim.x * wpb) {
    const uint32_t f = g * 64u + lane;
    const bool act = f < n;
    fdgpu_frag_ex_t x = act ? fx[f] : fdgpu_frag_ex_t{0u, 0u, 0u, 0u};
    const uint64_t line = (act && chk) ? chk[2u * f] : 0ull;
    const uint64_t seq = line ? chk[2u * f + 1u] : 0ull;
    if (rtab && act) {                                  /* DMA gather: the payload is in the arena already */
      x.off = (uint32_t)(rtab[x.sz >> 16] + x.off);
      x.sz &= 0xFFFFu;
    }
    const uint64_t s = (act && !rtab) ? src[f] : 0ull;
    const uint32_t nq = rtab ? 0u : (x.sz + 15u) >> 4;
    const uint32_t incl = wave_incl_scan(nq), excl = incl - nq;
    const uint32_t total = (uint32_t)__shfl((int)incl, 63, 64);
    /* unit k of the group: its owner lane's source and arena place (all
       lanes take part in the shuffles; a lane past the end reads the last
       unit's arena place instead of the bus, and stores nothing) */
    auto unit = [&](uint32_t k, const uint4 *&sp, uint4 *&dp) {
      const uint32_t kk = k < total ? k : total - 1u;
      const uint32_t o = unit_owner(incl, kk);
      const uint32_t u = kk - (uint32_t)__shfl((int)excl, (int)o, 64);
      sp = (const uint4 *)(uint64_t)__shfl((long long)s, (int)o, 64) + u;
      dp = (uint4 *)(arena + (uint32_t)__shfl((int)x.off, (int)o, 64)) + u;
      if (k >= total) sp = dp;
    };
    for (uint32_t k0 = 0; k0 < total; k0 += 256u) {
      const uint4 *s0, *s1, *s2, *s3;
      uint4 *d0, *d1, *d2, *d3;
      unit(k0 + lane, s0, d0);
      unit(k0 + 64u + lane, s1, d1);
      unit(k0 + 128u + lane, s2, d2);
      unit(k0 + 192u + lane, s3, d3);
      const uint4 v0 = *s0, v1 = *s1, v2 = *s2, v3 = *s3;       /* four loads over the bus in flight */
      if (k0 + lane < total) *d0 = v0;
      if (k0 + 64u + lane < total) *d1 = v1;
      if (k0 + 128u + lane < total) *d2 = v2;
      if (k0 + 192u + lane < total) *d3 = v3;
    }
    /* every payload load of the wave has returned (and every copy store is
       done: vmcnt counts both on gfx9) before a line is re-read */
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (line) {
      const uint64_t cur = __hip_atomic_load((const uint64_t *)line, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (cur != seq) x.tr_cap |= FDGPU_FX_LAPPED;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");      /* this CU's L1 holds none of the old arena bytes */
    uint32_t c = 0;
    fdgpu_txn_t dt{};
    if (act) {
      fx_dev[f] = x;
      fdt_txn_t *t = (fdt_txn_t *)(txn_out + (size_t)f * FDT_TXN_MAX_SZ);
      uint64_t why = 0;
      /* a lapped payload may be torn: not parsed */
      uint64_t fp = (x.tr_cap & FDGPU_FX_LAPPED) ? 0u : fdt_parse_core(arena + x.off, x.sz, t, &why);
      const uint32_t sc = fp ? t->signature_cnt : 0u;
      c = (sc >= 1u && sc <= 16u) ? sc : 0u;
      if (c > fdt_frag_sig_bound(x.sz)) { c = 0u; fp = 0u; }      /* cannot happen for a parsed txn */
      if (fp) {
        dt.msg_off = x.off + t->message_off;
        dt.msg_sz = x.sz - t->message_off;
        dt.sig_off = x.off + t->signature_off;
        dt.pub_off = x.off + t->acct_addr_off;
      }
      txn_sz[f] = (uint16_t)fp;
    }
    const uint32_t ci = wave_incl_scan(c);
    const uint32_t ct = (uint32_t)__shfl((int)ci, 63, 64);
    uint32_t base = 0;
    if (lane == 63u && ct) base = atomicAdd(n_sig, ct);
    base = (uint32_t)__shfl((int)base, 63, 64);
    if (!act) continue;
    const uint32_t s0 = base + ci - c;
    fdgpu_txn_desc_t td;
    td.sig0 = s0;
    td.sig_cnt = c;
    tds[f] = td;
    for (uint32_t j = 0; j < c; j++) {
      fdgpu_sig_desc_t sd;
      sd.msg_off = dt.msg_off;
      sd.msg_sz = dt.msg_sz;
      sd.sig_off = dt.sig_off + 64u * j;
      sd.pub_off = dt.pub_off + 32u * j;
      sigs[s0 + j] = sd;
    }
  }
}

/* bytes b, b+1 (b even) of a frag's out frag [payload sz][pad to 2]
   [fd_txn_t fp][u16 sz] as one 16-bit word: the payload (16-B aligned in
   the arena), the fd_txn_t (4-B aligned record, toff even) and the size
   word all split on even offsets, so every half is one aligned 2-B load */
FDG_DEV uint32_t out_frag_half(uint32_t b, const uint8_t *pl, uint32_t sz, uint32_t toff, const uint8_t *tr,
                               uint32_t fp) {
  if (b < toff) {
    const uint32_t v = *(const uint16_t *)(pl + b);
    return b + 1u < sz ? v : v & 0xffu;                 /* the pad byte of an odd payload */
  }
  if (b < toff + fp) return *(const uint16_t *)(tr + (b - toff));
  return b == toff + fp ? sz & 0xffffu : 0u;
}

/* Finish: per group, lane i writes frag i's code (the batch_single_msg
   combine of its signatures; FDGPU_CODE_PARSE_FAIL; FDGPU_CODE_LAPPED;
   FDGPU_CODE_TRAILER_CAP when the out frag would not fit the caller's
   reservation), its dedup tag (fd_hash of the first signature,
   fd_verify.h:66) and its out size (coalesced over the lanes); then the wave
   writes the group's out frags as fd_verify.c:93-136 lays them out in the
   out dcache -- [payload][pad to 2][fd_txn_t][u16 payload_sz] -- one 16-B
   unit per lane and step, the units flattened over the group: a unit inside
   the payload is one 16-B load from the arena, the others are assembled
   byte by byte; a unit that would pass the frag's reservation (or an out
   frag not 16-B aligned) is written in 2-B stores up to the frag's end.  The
   first thread clears the slot's ingest counter for its next gathered batch
   (zero_next; the verify that read it is complete).  (A completion word
   stored by the kernel's last block was tried: the system-scope fence each
   block then needs writes back the L2 under the concurrent verify kernels
   and halved the tile's rate; the stream's own write after the kernel
   stays.) */
__global__ void __launch_bounds__(256) fdgpu_frag_finish_io_kernel(
    const fdgpu_txn_desc_t *__restrict__ txns, uint32_t n, const int8_t *__restrict__ sig_codes,
    const uint16_t *__restrict__ txn_sz, const fdgpu_frag_ex_t *__restrict__ fx, const uint8_t *__restrict__ txn_out,
    const uint8_t *__restrict__ arena, uint64_t seed, uint8_t *__restrict__ out, int8_t *__restrict__ codes,
    uint64_t *__restrict__ tags, uint16_t *__restrict__ out_szs, uint32_t *__restrict__ zero_next) {
  const uint32_t lane = threadIdx.x & 63u, wpb = blockDim.x >> 6;
  if (blockIdx.x == 0 && threadIdx.x == 0 && zero_next) *zero_next = 0u;
  for (uint32_t g = blockIdx.x * wpb + (threadIdx.x >> 6); g * 64u < n; g += gridDim.x * wpb) {
    const uint32_t f = g * 64u + lane;
    const bool act = f < n;
    uint32_t fp = 0, osz = 0, toff = 0;
    fdgpu_frag_ex_t x{0u, 0u, 0u, 0u};            /* off: arena, sz, tr_off: out offset, tr_cap: its room */
    bool fits = false;
    if (act) {
      fp = txn_sz[f];
      x = fx[f];
      const bool lapped = (x.tr_cap & FDGPU_FX_LAPPED) != 0u;   /* fp is 0 then */
      toff = (x.sz + 1u) & ~1u;
      osz = toff + fp + 2u;
      fits = fp && osz <= x.tr_cap;
      const fdt_txn_t *t = (const fdt_txn_t *)(txn_out + (size_t)f * FDT_TXN_MAX_SZ);
      int code = lapped ? FDGPU_CODE_LAPPED : FDGPU_CODE_PARSE_FAIL;
      uint64_t tag = 0;
      if (fp) {
        tag = fdt_hash_core(seed, arena + x.off + t->signature_off, 64);
        if (!fits) {
          code = FDGPU_CODE_TRAILER_CAP;
        } else {
          code = -1;
          const fdgpu_txn_desc_t d = txns[f];
          if (d.sig_cnt >= 1 && d.sig_cnt <= 16) {           /* else ERR_SIG (fd_ed25519_user.c:238-241) */
            int first_struct = 0, any_msg = 0;
            for (uint32_t j = 0; j < d.sig_cnt; j++) {
              const int c = sig_codes[d.sig0 + j];
              if (c == -3) any_msg = 1;
              else if (c != 0 && first_struct == 0) first_struct = c;
            }
            code = first_struct ? first_struct : (any_msg ? -3 : 0);
          }
        }
      }
      codes[f] = (int8_t)code;
      tags[f] = tag;
      out_szs[f] = (uint16_t)(fits ? osz : 0u);
    }
    const uint32_t nu = fits ? (osz + 15u) >> 4 : 0u;
    const uint32_t incl = wave_incl_scan(nu), excl = incl - nu;
    const uint32_t total = (uint32_t)__shfl((int)incl, 63, 64);
    for (uint32_t k0 = 0; k0 < total; k0 += 64u) {       /* wave-uniform: every lane takes part in the shuffles */
      const uint32_t k = k0 + lane < total ? k0 + lane : total - 1u;
      const uint32_t o = unit_owner(incl, k);
      const uint32_t u = k - (uint32_t)__shfl((int)excl, (int)o, 64);
      const uint32_t off = (uint32_t)__shfl((int)x.off, (int)o, 64), sz = (uint32_t)__shfl((int)x.sz, (int)o, 64);
      const uint32_t oof = (uint32_t)__shfl((int)x.tr_off, (int)o, 64);
      const uint32_t cap = (uint32_t)__shfl((int)x.tr_cap, (int)o, 64) & 0xFFFFu;
      const uint32_t ofp = (uint32_t)__shfl((int)fp, (int)o, 64), oosz = (uint32_t)__shfl((int)osz, (int)o, 64);
      const uint32_t otoff = (sz + 1u) & ~1u, b0 = 16u * u;
      const uint8_t *pl = arena + off;
      const uint8_t *tr = txn_out + (size_t)(g * 64u + o) * FDT_TXN_MAX_SZ;
      uint8_t *dst = out + oof + b0;
      if (k0 + lane >= total) continue;
      if (b0 + 16u <= cap && !(((uintptr_t)dst) & 15u)) {
        uint4 w;
        if (b0 + 16u <= sz) {
          w = *(const uint4 *)(pl + b0);                      /* arena offsets are 16-B aligned */
        } else {
          uint32_t q[4];
#pragma unroll
          for (int i = 0; i < 4; i++)
            q[i] = out_frag_half(b0 + 4u * i, pl, sz, otoff, tr, ofp) |
                   (out_frag_half(b0 + 4u * i + 2u, pl, sz, otoff, tr, ofp) << 16);
          w = make_uint4(q[0], q[1], q[2], q[3]);
        }
        *(uint4 *)dst = w;
      } else {
        for (uint32_t b = b0; b < b0 + 16u && b < oosz; b += 2u)
          *(uint16_t *)(out + oof + b) = (uint16_t)out_frag_half(b, pl, sz, otoff, tr, ofp);
      }
    }
  }
}

/* After the combine: a payload that did not parse gets FDGPU_CODE_PARSE_FAIL */
__global__ void __launch_bounds__(256) fdgpu_frag_codes_kernel(const uint16_t *__restrict__ txn_sz, uint32_t n,
                                                               int8_t *__restrict__ codes) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n && !txn_sz[t]) codes[t] = (int8_t)FDGPU_CODE_PARSE_FAIL;
}

/* hs_split on the device (v_rcp_f64 quotients) for the parity tests: n
   scalars k < L (8 words each) -> 16 words each: |u| (5), |v| (5), ok,
   u_neg, v_neg, bits, 0, 0 */
__global__ void __launch_bounds__(64) fdgpu_test_hs_split_kernel(const uint32_t *in, uint32_t *out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t k[8];
  for (int j = 0; j < 8; j++) k[j] = i < n ? in[8 * i + j] : 0u;
  hs_split_t o;
  hs_split(o, k);                               /* every lane runs it: the loops are wave-uniform */
  if (i >= n) return;
  uint32_t *w = out + 16 * (size_t)i;
  for (int j = 0; j < 5; j++) { w[j] = o.u[j]; w[5 + j] = o.v[j]; }
  w[10] = o.ok; w[11] = o.u_neg; w[12] = o.v_neg; w[13] = o.bits; w[14] = 0u; w[15] = 0u;
}

}  // namespace

extern "C" {

char const *fdgpu_kernel_path(void) { return "halfsize: fdgpu_verify_hs_kernel + fdgpu_full_kernel"; }

#ifndef FDGPU_PHASE_STAMPS
#define FDGPU_PHASE_STAMPS 0
#endif
/* every compile-time switch of the kernels, as JSON members; the return
   value is 1 iff each is at the shipped default (fdgpu_build_info) */
int fdgpu_kernel_build_info(char *buf, size_t n) {
  snprintf(buf, n, "\"verify_waves\":%d,\"atab_words\":%u,\"tab_store_nt\":%d,\"tab_load_cpol\":%d,\"ws_slot\":%d,"
           "\"phase_stamps\":%d", (int)FDGPU_VERIFY_WAVES, (unsigned)FDGPU_ATAB_WORDS, (int)FDGPU_TAB_STORE_NT,
           (int)FDGPU_TAB_LOAD_CPOL, (int)FDGPU_WS_SLOT, (int)FDGPU_PHASE_STAMPS);
  return FDGPU_VERIFY_WAVES == 2 && FDGPU_ATAB_WORDS == 40u && FDGPU_TAB_STORE_NT == 0 && FDGPU_TAB_LOAD_CPOL == 0 &&
         FDGPU_WS_SLOT == 0 && FDGPU_PHASE_STAMPS == 0;
}

size_t fdgpu_btab_bytes(void) {
  return (BTAB_WORDS + (FDGPU_WS_SLOT ? FDGPU_WS_SLOTS / 32u + (size_t)FDGPU_WS_SLOTS * 64u * FDGPU_WS_LANE_WORDS : 0)) *
         sizeof(uint32_t);
}

hipError_t fdgpu_btab_build(uint32_t *d_btab, hipStream_t stream) {
  uint32_t *bases = nullptr, *scratch = nullptr;
  const uint32_t lanes = BC_NDIG * BC_CHUNKS;
  hipError_t e = FDGPU_WS_SLOT ? hipMemsetAsync(d_btab + BTAB_WORDS, 0, FDGPU_WS_SLOTS / 8u, stream) : hipSuccess;
  if (e == hipSuccess) e = hipMalloc((void **)&bases, BC_NDIG * 40 * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc((void **)&scratch, (size_t)lanes * FDGPU_BCOMB_CHUNK * 10 * sizeof(uint32_t));
  if (e == hipSuccess) {
    hipLaunchKernelGGL(fdgpu_bcomb_base_kernel, dim3(1), dim3(64), 0, stream, bases);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(fdgpu_bcomb_fill_kernel, dim3((lanes + 63) / 64), dim3(64), 0, stream, bases, d_btab, scratch);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  if (bases) (void)hipFree(bases);
  if (scratch) (void)hipFree(scratch);
  return e;
}

hipError_t fdgpu_verify_occupancy(int *blocks_per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fdgpu_verify_hs_kernel<false>, FDGPU_BLOCK, 0);
}

/* workspace: per-lane words, the fallback queue, its counter and the key
   cache's representative count (16 words), then the key cache's hash table,
   key_of, verdicts and representative list */
static uint64_t kc_ht_slots(uint64_t lanes) {       /* power of two >= 2 lanes */
  uint64_t h = 64;
  while (h < 2 * lanes) h <<= 1;
  return h;
}

size_t fdgpu_ws_bytes(uint64_t n_sig) {
  const uint64_t grid = (n_sig + FDGPU_BLOCK - 1) / FDGPU_BLOCK, lanes = grid * FDGPU_BLOCK;
  return (size_t)(lanes * FDGPU_WS_LANE_WORDS + lanes + 16 + kc_ht_slots(lanes) + 3 * lanes) * sizeof(uint32_t);
}

hipError_t fdgpu_launch_verify_sigs(const uint8_t *d_arena, const fdgpu_sig_desc_t *d_sigs, uint32_t n_sig,
                                    const uint32_t *d_perm, const uint32_t *d_btab, uint32_t *d_ws,
                                    int8_t *d_sig_codes, uint32_t flags, hipStream_t stream, const uint32_t *d_n_sig,
                                    uint32_t resident_blocks, uint64_t kc_seed, int cnt_zeroed) {
  if (!n_sig) return hipSuccess;
  const uint32_t grid = (n_sig + FDGPU_BLOCK - 1) / FDGPU_BLOCK;
  const size_t lanes = (size_t)grid * FDGPU_BLOCK;
  uint32_t *queue = d_ws + lanes * FDGPU_WS_LANE_WORDS, *cnt = queue + lanes;
  hipError_t e = cnt_zeroed ? hipSuccess : hipMemsetAsync(cnt, 0, sizeof(uint32_t), stream);
  if (e != hipSuccess) return e;
  /* the queued full-length lanes get as many blocks as the batch's grid could
     keep resident (all of them, up to every wave slot of the GPU: the
     engine's occupancy x CUs), each exiting at once when the queue holds
     nothing for it */
  if (!resident_blocks) resident_blocks = 1;
  uint32_t slow_blocks = grid < resident_blocks ? grid : resident_blocks;
  /* strides over its queue; a tile-sized batch (<= 64 blocks) gets a quarter */
  const uint32_t slow_cap = grid > 64u ? FDGPU_FULL_BLOCKS : FDGPU_FULL_BLOCKS / 4u;
  if (slow_blocks > slow_cap) slow_blocks = slow_cap;
  const uint32_t *key_of = nullptr;
  if (flags & FDGPU_FLAG_KCACHE) {
    const uint64_t hts = kc_ht_slots(lanes);
    uint32_t *ht = cnt + 16, *kof = ht + hts, *kverd = kof + lanes, *reps = kverd + lanes, *rep_cnt = cnt + 1;
    e = hipMemsetAsync(ht, 0xff, hts * sizeof(uint32_t), stream);
    if (e == hipSuccess) e = hipMemsetAsync(rep_cnt, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(fdgpu_key_dedup_kernel, dim3((n_sig + 255) / 256), dim3(256), 0, stream, d_arena, d_sigs, n_sig,
                       d_n_sig, ht, (uint32_t)(hts - 1), kof, reps, rep_cnt, kc_seed);
    hipLaunchKernelGGL(fdgpu_key_table_kernel, dim3(grid), dim3(FDGPU_BLOCK), 0, stream, d_arena, d_sigs, d_ws, reps,
                       rep_cnt, kverd, flags);
    hipLaunchKernelGGL(fdgpu_verify_hs_kernel<true>, dim3(grid), dim3(FDGPU_BLOCK), 0, stream, d_arena, d_sigs, n_sig,
                       d_n_sig, d_btab, d_ws, d_perm, d_sig_codes, queue, cnt, flags, kof, kverd);
    key_of = kof;
  } else if (flags & FDGPU_FLAG_KPAIR) {
    const uint32_t pgrid = (2u * n_sig + FDGPU_BLOCK - 1) / FDGPU_BLOCK;     /* two lanes per signature */
    hipLaunchKernelGGL(fdgpu_verify_pair_kernel, dim3(pgrid), dim3(FDGPU_BLOCK),
                       (flags & FDGPU_FLAG_KSPREAD) ? FDGPU_SPREAD_LDS_PAIR : 0, stream, d_arena, d_sigs, n_sig,
                       d_n_sig, d_btab, d_ws, d_perm, d_sig_codes, queue, cnt, flags);
  } else {
    hipLaunchKernelGGL(fdgpu_verify_hs_kernel<false>, dim3(grid), dim3(FDGPU_BLOCK),
                       (flags & FDGPU_FLAG_KSPREAD) ? FDGPU_SPREAD_LDS : 0, stream, d_arena, d_sigs, n_sig,
                       d_n_sig, d_btab, d_ws, d_perm, d_sig_codes, queue, cnt, flags, nullptr, nullptr);
  }
  hipLaunchKernelGGL(fdgpu_full_kernel, dim3(slow_blocks), dim3(FDGPU_BLOCK), 0, stream, d_ws, d_perm, d_sig_codes,
                     queue, cnt, slow_blocks * FDGPU_BLOCK, key_of);
  return hipGetLastError();
}

uint64_t fdgpu_sha512_stream_blocks(uint64_t msg_sz) { return (64u + msg_sz + 16u) / 128u + 1u; }

hipError_t fdgpu_launch_sha512_stream(const uint8_t *d_mbuf, uint64_t m0, uint64_t mlen, uint64_t msg_sz,
                                      uint64_t blk0, uint32_t nblk, const uint8_t *d_ra, uint64_t *d_state,
                                      uint32_t n, hipStream_t stream) {
  if (!n || n > 64 || !nblk) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fdgpu_sha512_stream_kernel, dim3(1), dim3(64), 0, stream, d_mbuf, m0, mlen, msg_sz, blk0, nblk,
                     d_ra, d_state, n);
  return hipGetLastError();
}

hipError_t fdgpu_launch_verify_prehashed(const uint8_t *d_arena, const fdgpu_sig_desc_t *d_sigs, uint32_t n_sig,
                                         const uint32_t *d_btab, uint32_t *d_ws, int8_t *d_sig_codes, uint32_t flags,
                                         hipStream_t stream) {
  if (!n_sig) return hipSuccess;
  const uint32_t grid = (n_sig + FDGPU_BLOCK - 1) / FDGPU_BLOCK;
  const size_t lanes = (size_t)grid * FDGPU_BLOCK;
  uint32_t *queue = d_ws + lanes * FDGPU_WS_LANE_WORDS, *cnt = queue + lanes;
  hipError_t e = hipMemsetAsync(cnt, 0, sizeof(uint32_t), stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((fdgpu_verify_hs_kernel<false, true>), dim3(grid), dim3(FDGPU_BLOCK), 0, stream, d_arena, d_sigs,
                     n_sig, nullptr, d_btab, d_ws, nullptr, d_sig_codes, queue, cnt, flags & FDGPU_FLAG_REF_MAP,
                     nullptr, nullptr);
  hipLaunchKernelGGL(fdgpu_full_kernel, dim3(1), dim3(FDGPU_BLOCK), 0, stream, d_ws, nullptr, d_sig_codes, queue, cnt,
                     FDGPU_BLOCK, nullptr);
  return hipGetLastError();
}

hipError_t fdgpu_launch_verify_multi(const fdgpu_mbatch_t *mb, uint32_t nb, uint32_t grid_max, uint32_t slow_max,
                                     const uint32_t *d_btab, uint32_t flags, hipStream_t stream) {
  if (!nb || !grid_max) return hipSuccess;
  hipLaunchKernelGGL(fdgpu_verify_hs_multi_kernel, dim3(grid_max, nb), dim3(FDGPU_BLOCK), 0, stream, mb, d_btab, flags);
  hipLaunchKernelGGL(fdgpu_full_multi_kernel, dim3(slow_max ? slow_max : 1, nb), dim3(FDGPU_BLOCK), 0, stream, mb);
  return hipGetLastError();
}

uint32_t *fdgpu_verify_cnt_word(uint32_t *d_ws, uint32_t n_sig) {
  const size_t lanes = (size_t)((n_sig + FDGPU_BLOCK - 1) / FDGPU_BLOCK) * FDGPU_BLOCK;
  return d_ws + lanes * FDGPU_WS_LANE_WORDS + lanes;
}

hipError_t fdgpu_launch_combine(const fdgpu_txn_desc_t *d_txns, uint32_t n_txn, const int8_t *d_sig_codes,
                                int8_t *d_txn_codes, uint64_t *d_accept, hipStream_t stream) {
  if (!n_txn) return hipSuccess;
  const uint32_t blocks = (n_txn + 255) / 256;
  hipLaunchKernelGGL(fdgpu_combine_kernel, dim3(blocks < FDGPU_AUX_BLOCKS ? blocks : FDGPU_AUX_BLOCKS), dim3(256), 0,
                     stream, d_txns, n_txn, d_sig_codes, d_txn_codes, d_accept);
  return hipGetLastError();
}

#if FDGPU_PHASE_STAMPS
/* diagnostic builds: copy out the per-wave phase stamps */
int fdgpu_debug_stamps(uint64_t *out, uint64_t n_waves) {
  if (n_waves > FDGPU_STAMP_WAVES) n_waves = FDGPU_STAMP_WAVES;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fdgpu_stamps), n_waves * FDGPU_STAMP_SLOTS * sizeof(uint64_t)) ==
                 hipSuccess ? 0 : -1;
}
#endif

hipError_t fdgpu_launch_test_fe(const uint32_t *d_in, uint32_t *d_out, uint32_t n, hipStream_t stream) {
  hipLaunchKernelGGL(fdgpu_test_fe_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, d_in, d_out, n);
  return hipGetLastError();
}
hipError_t fdgpu_launch_test_decode(const uint32_t *d_enc, uint32_t *d_out, uint32_t n, uint32_t flags,
                                    hipStream_t stream) {
  hipLaunchKernelGGL(fdgpu_test_decode_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, d_enc, d_out, n, flags);
  return hipGetLastError();
}
hipError_t fdgpu_launch_test_sha512(const uint8_t *d_arena, const fdgpu_sig_desc_t *d_msgs, uint32_t n,
                                    uint32_t *d_out, hipStream_t stream) {
  hipLaunchKernelGGL(fdgpu_test_sha512_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, d_arena, d_msgs, n, d_out);
  return hipGetLastError();
}
hipError_t fdgpu_launch_test_hram(const uint8_t *d_arena, const fdgpu_sig_desc_t *d_sigs, uint32_t n,
                                  uint32_t *d_out, hipStream_t stream) {
  hipLaunchKernelGGL(fdgpu_test_hram_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, d_arena, d_sigs, n, d_out);
  return hipGetLastError();
}
hipError_t fdgpu_launch_test_sc_reduce(const uint32_t *d_in, uint32_t *d_out, uint32_t n, hipStream_t stream) {
  hipLaunchKernelGGL(fdgpu_test_sc_reduce_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, d_in, d_out, n);
  return hipGetLastError();
}
uint64_t fdgpu_frag_sig_bound(uint32_t sz) { return fdt_frag_sig_bound(sz); }

hipError_t fdgpu_launch_frag_ingest(const uint8_t *d_arena, const void *d_frags, uint32_t frag_stride, uint32_t n,
                                    uint8_t *d_txn_out, uint16_t *d_txn_sz, fdgpu_txn_t *d_txd, uint32_t *d_cnt,
                                    uint32_t *d_sig0, uint32_t *d_blocktot, uint32_t *d_n_sig,
                                    fdgpu_sig_desc_t *d_sigs, fdgpu_txn_desc_t *d_tds, hipStream_t stream) {
  if (!n) return hipMemsetAsync(d_n_sig, 0, sizeof(uint32_t), stream);
  const uint32_t nb = (n + FDGPU_SCAN_BLOCK - 1) / FDGPU_SCAN_BLOCK;
  hipLaunchKernelGGL(fdgpu_frag_parse_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, d_arena,
                     (const uint32_t *)d_frags, frag_stride, n, d_txn_out,
                     d_txn_sz, d_txd, d_cnt);
  hipLaunchKernelGGL(fdgpu_scan_local_kernel, dim3(nb), dim3(256), 0, stream, d_cnt, n, d_sig0, d_blocktot);
  hipLaunchKernelGGL(fdgpu_scan_blocks_kernel, dim3(1), dim3(1024), 0, stream, d_blocktot, nb, d_n_sig);
  hipLaunchKernelGGL(fdgpu_frag_expand_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, d_txd, d_cnt, d_sig0,
                     d_blocktot, n, d_sigs, d_tds);
  return hipGetLastError();
}

hipError_t fdgpu_launch_frag_codes(const uint16_t *d_txn_sz, uint32_t n, int8_t *d_codes, hipStream_t stream) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(fdgpu_frag_codes_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, d_txn_sz, n, d_codes);
  return hipGetLastError();
}

hipError_t fdgpu_launch_frag_ring(const uint8_t *d_arena, const fdgpu_frag_ex_t *d_fx, uint32_t n, uint8_t *d_txn_out,
                                  uint16_t *d_txn_sz, fdgpu_txn_t *d_txd, uint32_t *d_cnt, uint32_t *d_sig0,
                                  uint32_t *d_blocktot, uint32_t *d_n_sig, fdgpu_sig_desc_t *d_sigs,
                                  fdgpu_txn_desc_t *d_tds, hipStream_t stream) {
  if (!n) return hipMemsetAsync(d_n_sig, 0, sizeof(uint32_t), stream);
  if (n > FDGPU_SMALL_SCAN_MAX)
    return fdgpu_launch_frag_ingest(d_arena, d_fx, 4u, n, d_txn_out, d_txn_sz, d_txd, d_cnt, d_sig0, d_blocktot,
                                    d_n_sig, d_sigs, d_tds, stream);
  hipLaunchKernelGGL(fdgpu_frag_parse_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, d_arena,
                     (const uint32_t *)d_fx, 4u, n, d_txn_out, d_txn_sz, d_txd, d_cnt);
  hipLaunchKernelGGL(fdgpu_frag_scan_expand_small_kernel, dim3(1), dim3(1024), 0, stream, d_txd, d_cnt, n, d_sigs,
                     d_tds, d_n_sig);
  return hipGetLastError();
}

hipError_t fdgpu_launch_frag_finish(const fdgpu_txn_desc_t *d_tds, uint32_t n, const int8_t *d_sig_codes,
                                    const uint16_t *d_txn_sz, const fdgpu_frag_ex_t *d_fx, const uint8_t *d_txn_out,
                                    int8_t *d_codes, uint8_t *d_trailers, hipStream_t stream) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(fdgpu_frag_finish_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, d_tds, n, d_sig_codes,
                     d_txn_sz, d_fx, d_txn_out, d_codes, d_trailers);
  return hipGetLastError();
}

uint64_t fdgpu_frag_fp_bound(uint32_t sz) { return fdt_frag_fp_bound(sz); }

static uint32_t env_u32(const char *k, uint32_t d) {
  const char *v = getenv(k);
  return v && atoi(v) > 0 ? (uint32_t)atoi(v) : d;
}
static const uint32_t g_aux_in = env_u32("FDGPU_AUX_BLOCKS_IN", FDGPU_IO_BLOCKS);
static const uint32_t g_aux_fin = env_u32("FDGPU_AUX_BLOCKS_FIN", FDGPU_IO_BLOCKS);
static uint32_t aux_blocks(uint32_t n, uint32_t cap = FDGPU_AUX_BLOCKS) {   /* waves of 64 frags, 4 per block */
  const uint32_t b = (n + 255u) / 256u;
  return b < cap ? b : cap;
}

hipError_t fdgpu_launch_frag_ingest_io(const uint64_t *d_src, const fdgpu_frag_ex_t *d_fx, const uint64_t *d_chk,
                                       const uint64_t *d_rtab, uint32_t n, uint8_t *d_arena,
                                       fdgpu_frag_ex_t *d_fx_dev, uint8_t *d_txn_out, uint16_t *d_txn_sz,
                                       fdgpu_sig_desc_t *d_sigs, fdgpu_txn_desc_t *d_tds, uint32_t *d_n_sig,
                                       uint32_t *d_zero_word, hipStream_t stream) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(fdgpu_frag_ingest_io_kernel, dim3(aux_blocks(n, g_aux_in)), dim3(256), 0, stream, d_src, d_fx, d_chk,
                     d_rtab, n, d_arena, d_fx_dev, d_txn_out, d_txn_sz, d_sigs, d_tds, d_n_sig, d_zero_word);
  return hipGetLastError();
}

hipError_t fdgpu_launch_frag_finish_io(const fdgpu_txn_desc_t *d_tds, uint32_t n, const int8_t *d_sig_codes,
                                       const uint16_t *d_txn_sz, const fdgpu_frag_ex_t *d_fx, const uint8_t *d_txn_out,
                                       const uint8_t *d_arena, uint64_t hash_seed, uint8_t *d_out, int8_t *d_codes,
                                       uint64_t *d_tags, uint16_t *d_out_szs, uint32_t *d_zero_next,
                                       hipStream_t stream) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(fdgpu_frag_finish_io_kernel, dim3(aux_blocks(n, g_aux_fin)), dim3(256), 0, stream, d_tds, n, d_sig_codes,
                     d_txn_sz, d_fx, d_txn_out, d_arena, hash_seed, d_out, d_codes, d_tags, d_out_szs, d_zero_next);
  return hipGetLastError();
}

hipError_t fdgpu_launch_test_hs_split(const uint32_t *d_in, uint32_t *d_out, uint32_t n, hipStream_t stream) {
  hipLaunchKernelGGL(fdgpu_test_hs_split_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, d_in, d_out, n);
  return hipGetLastError();
}

}  // extern "C"
