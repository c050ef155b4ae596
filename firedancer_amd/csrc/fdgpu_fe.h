/* fdgpu_fe.h -- GF(2^255-19) arithmetic for one field element per lane on
   gfx950 (MI355X), radix 2^25.5: 10 unsigned 32-bit limbs, limb i has
   weight 2^(25 i + ceil(i/2)) (widths 26,25,26,...,25; 255 bits in all).

   Why this representation (tools/ubench_int.hip, tools/ubench_fe.hip, run on
   MI355X, profiles/r01_ubench_int.jsonl and r01_ubench_fe.jsonl): every 32-bit integer multiply form on
   gfx950 issues at half rate (~61 lane-ops/CU/clk) and so do VOP3 adds with
   a carry-out, while plain v_add_u32/v_mov_b32 issue at full rate.  Radix
   2^25.5 needs no carries inside a product (64-bit column sums), makes
   add/sub carry-free limb-wise v_add_u32 (full rate), and measured as fast
   as the best radix-2^32 variant (inline-asm v_mad_u64_u32 carry chains)
   for mul alone.

   Bounds discipline (all values are non-negative limb vectors, any
   representative of the residue class):
     R  (reduced)  limbs <= 2^26 (+2^17.2 on limbs 1,5)     mul/sq/carry outputs
     A  (added)    R + R         limbs <= 2^27
     S  (sub 2p)   R + 2p - R    limbs <= 2^26 + 2^27
     S4 (sub 4p)   x + 4p - y    limbs <= 2^26 + 2^28      (y up to A)
   fe_mul(f, g) is exact when 2 f_i < 2^32, 19 g_j < 2^32 (g limbs < 2^27.75)
   and 267 * max(f) * max(g) < 2^64 (267 = largest column coefficient sum):
     R, A, S are valid for both operands; S4 only as the FIRST operand with
     the second at most A.  Every call site in fdgpu_ge.h is annotated.

   Restates the field layer of the reference (avx512/fd_f25519.h,
   avx512/fd_r43x6.h:754-1025 mul/sqr, fd_r43x6.c:98-148 pow22523,
   fd_r43x6.h:1117-1128 diagnose) in a different, GPU-native
   representation; only observable values (canonical residues) must match. */
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fdgpu_consts.h"

#define FDG_DEV __device__ __forceinline__

/* Scheduling fence after each multiply: stops the machine scheduler from
   interleaving consecutive independent field products (which it otherwise
   does up to the full VGPR budget, forcing spills in the point formulas).
   Each product alone has 10 independent column chains of ILP. */
#define FDG_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

namespace fdgpu {

struct fe { uint32_t v[10]; };

template <int I> struct limb_w { static constexpr int bits = (I & 1) ? 25 : 26; };

FDG_DEV void fe_set(fe &h, const uint32_t (&c)[10]) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = c[i];
}
FDG_DEV void fe_0(fe &h) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = 0;
}
FDG_DEV void fe_1(fe &h) { fe_0(h); h.v[0] = 1; }

/* h = f + g  (R,R -> A) */
FDG_DEV void fe_add(fe &h, const fe &f, const fe &g) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = f.v[i] + g.v[i];
}

/* h = f - g = f + 2p - g  (g must be <= R; output S) */
FDG_DEV void fe_sub(fe &h, const fe &f, const fe &g) {
  constexpr uint32_t P2[10] = FDGPU_FE_2P;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = f.v[i] + P2[i] - g.v[i];
}

/* h = f - g = f + 4p - g  (g up to A; output S4) */
FDG_DEV void fe_sub4(fe &h, const fe &f, const fe &g) {
  constexpr uint32_t P4[10] = FDGPU_FE_4P;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = f.v[i] + P4[i] - g.v[i];
}

/* h = -f = 2p - f  (f <= R; output <= 2^27) */
FDG_DEV void fe_neg(fe &h, const fe &f) {
  constexpr uint32_t P2[10] = FDGPU_FE_2P;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = P2[i] - f.v[i];
}

/* Conditional select h = c ? a : b (per lane, branch-free). */
FDG_DEV void fe_cmov(fe &h, const fe &a, const fe &b, bool c) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = c ? a.v[i] : b.v[i];
}

/* Weak reduction of 32-bit limbs (inputs up to ~2^31) to R. */
FDG_DEV void fe_carry(fe &h) {
  constexpr uint32_t M26 = (1u << 26) - 1, M25 = (1u << 25) - 1;
  uint32_t t;
  t = h.v[0] >> 26; h.v[0] &= M26; h.v[1] += t;
  t = h.v[4] >> 26; h.v[4] &= M26; h.v[5] += t;
  t = h.v[1] >> 25; h.v[1] &= M25; h.v[2] += t;
  t = h.v[5] >> 25; h.v[5] &= M25; h.v[6] += t;
  t = h.v[2] >> 26; h.v[2] &= M26; h.v[3] += t;
  t = h.v[6] >> 26; h.v[6] &= M26; h.v[7] += t;
  t = h.v[3] >> 25; h.v[3] &= M25; h.v[4] += t;
  t = h.v[7] >> 25; h.v[7] &= M25; h.v[8] += t;
  t = h.v[4] >> 26; h.v[4] &= M26; h.v[5] += t;
  t = h.v[8] >> 26; h.v[8] &= M26; h.v[9] += t;
  t = h.v[9] >> 25; h.v[9] &= M25; h.v[0] += t * 19u;
  t = h.v[0] >> 26; h.v[0] &= M26; h.v[1] += t;
}

/* One parallel carry pass (every limb's excess moves up once, limb 9's
   wraps into limb 0 times 19): inputs up to 2^31 come out with limbs <=
   mask + 2^6 (limb 0: 2^26 + 19 * 2^6), inside R.  The ten steps are
   independent, 3 instructions each (fe_carry's sequential 12-step chain
   is 36 and serial). */
FDG_DEV void fe_carry_par(fe &h) {
  uint32_t c[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int w = (i & 1) ? 25 : 26;
    c[i] = h.v[i] >> w;
    h.v[i] &= (1u << w) - 1;
  }
  h.v[0] += 19u * c[9];
#pragma unroll
  for (int i = 1; i < 10; i++) h.v[i] += c[i - 1];
}

/* Column sums (tools/ubench_carry.hip, profiles/r01_ubench_carry.json): the
   columns are summed in order 0..9 and each column's v_mad_u64_u32 chain
   starts from the previous column's carry, so the carry add rides in a mad
   addend instead of a separate 64-bit add (the chain is kept in inline asm:
   the compiler would otherwise re-associate it into independent partial sums
   plus an add).  8% faster per product on gfx950 than ten independent column
   sums and a 12-step two-chain carry.  Outputs are R-bound (slack on limb 1
   only) and h is written last, so h may alias f or g.

   Each column's v_mad_u64_u32 chain is ONE inline-asm block.  With one
   block per mad the compiler's hazard recognizer cannot see inside the asm
   and pads every block with an s_nop; compiler-generated
   back-to-back mads writing the same carry SGPR need none, so a block of N
   dependent mads is as safe as N separate ones.  madc<N>::run(s, a, b):
   s += a[0] b[0] + ... + a[N-1] b[N-1], in that order. */
template <int N> struct madc;
template <> struct madc<1> {
  static FDG_DEV void run(uint64_t &s, const uint32_t *a, const uint32_t *b) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n"
        : "+v"(s), "=&s"(cc) : "v"(a[0]), "v"(b[0]));
    (void)cc;
  }
};
template <> struct madc<2> {
  static FDG_DEV void run(uint64_t &s, const uint32_t *a, const uint32_t *b) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n" "v_mad_u64_u32 %0, %1, %4, %5, %0\n"
        : "+v"(s), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(a[1]), "v"(b[1]));
    (void)cc;
  }
};
template <> struct madc<3> {
  static FDG_DEV void run(uint64_t &s, const uint32_t *a, const uint32_t *b) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n" "v_mad_u64_u32 %0, %1, %4, %5, %0\n" "v_mad_u64_u32 %0, %1, %6, %7, %0\n"
        : "+v"(s), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(a[1]), "v"(b[1]), "v"(a[2]), "v"(b[2]));
    (void)cc;
  }
};
template <> struct madc<4> {
  static FDG_DEV void run(uint64_t &s, const uint32_t *a, const uint32_t *b) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n" "v_mad_u64_u32 %0, %1, %4, %5, %0\n" "v_mad_u64_u32 %0, %1, %6, %7, %0\n" "v_mad_u64_u32 %0, %1, %8, %9, %0\n"
        : "+v"(s), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(a[1]), "v"(b[1]), "v"(a[2]), "v"(b[2]), "v"(a[3]), "v"(b[3]));
    (void)cc;
  }
};
template <> struct madc<5> {
  static FDG_DEV void run(uint64_t &s, const uint32_t *a, const uint32_t *b) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n" "v_mad_u64_u32 %0, %1, %4, %5, %0\n" "v_mad_u64_u32 %0, %1, %6, %7, %0\n" "v_mad_u64_u32 %0, %1, %8, %9, %0\n" "v_mad_u64_u32 %0, %1, %10, %11, %0\n"
        : "+v"(s), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(a[1]), "v"(b[1]), "v"(a[2]), "v"(b[2]), "v"(a[3]), "v"(b[3]), "v"(a[4]), "v"(b[4]));
    (void)cc;
  }
};
template <> struct madc<6> {
  static FDG_DEV void run(uint64_t &s, const uint32_t *a, const uint32_t *b) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n" "v_mad_u64_u32 %0, %1, %4, %5, %0\n" "v_mad_u64_u32 %0, %1, %6, %7, %0\n" "v_mad_u64_u32 %0, %1, %8, %9, %0\n" "v_mad_u64_u32 %0, %1, %10, %11, %0\n" "v_mad_u64_u32 %0, %1, %12, %13, %0\n"
        : "+v"(s), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(a[1]), "v"(b[1]), "v"(a[2]), "v"(b[2]), "v"(a[3]), "v"(b[3]), "v"(a[4]), "v"(b[4]), "v"(a[5]), "v"(b[5]));
    (void)cc;
  }
};
template <> struct madc<7> {
  static FDG_DEV void run(uint64_t &s, const uint32_t *a, const uint32_t *b) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n" "v_mad_u64_u32 %0, %1, %4, %5, %0\n" "v_mad_u64_u32 %0, %1, %6, %7, %0\n" "v_mad_u64_u32 %0, %1, %8, %9, %0\n" "v_mad_u64_u32 %0, %1, %10, %11, %0\n" "v_mad_u64_u32 %0, %1, %12, %13, %0\n" "v_mad_u64_u32 %0, %1, %14, %15, %0\n"
        : "+v"(s), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(a[1]), "v"(b[1]), "v"(a[2]), "v"(b[2]), "v"(a[3]), "v"(b[3]), "v"(a[4]), "v"(b[4]), "v"(a[5]), "v"(b[5]), "v"(a[6]), "v"(b[6]));
    (void)cc;
  }
};
template <> struct madc<8> {
  static FDG_DEV void run(uint64_t &s, const uint32_t *a, const uint32_t *b) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n" "v_mad_u64_u32 %0, %1, %4, %5, %0\n" "v_mad_u64_u32 %0, %1, %6, %7, %0\n" "v_mad_u64_u32 %0, %1, %8, %9, %0\n" "v_mad_u64_u32 %0, %1, %10, %11, %0\n" "v_mad_u64_u32 %0, %1, %12, %13, %0\n" "v_mad_u64_u32 %0, %1, %14, %15, %0\n" "v_mad_u64_u32 %0, %1, %16, %17, %0\n"
        : "+v"(s), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(a[1]), "v"(b[1]), "v"(a[2]), "v"(b[2]), "v"(a[3]), "v"(b[3]), "v"(a[4]), "v"(b[4]), "v"(a[5]), "v"(b[5]), "v"(a[6]), "v"(b[6]), "v"(a[7]), "v"(b[7]));
    (void)cc;
  }
};
template <> struct madc<9> {
  static FDG_DEV void run(uint64_t &s, const uint32_t *a, const uint32_t *b) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n" "v_mad_u64_u32 %0, %1, %4, %5, %0\n" "v_mad_u64_u32 %0, %1, %6, %7, %0\n" "v_mad_u64_u32 %0, %1, %8, %9, %0\n" "v_mad_u64_u32 %0, %1, %10, %11, %0\n" "v_mad_u64_u32 %0, %1, %12, %13, %0\n" "v_mad_u64_u32 %0, %1, %14, %15, %0\n" "v_mad_u64_u32 %0, %1, %16, %17, %0\n" "v_mad_u64_u32 %0, %1, %18, %19, %0\n"
        : "+v"(s), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(a[1]), "v"(b[1]), "v"(a[2]), "v"(b[2]), "v"(a[3]), "v"(b[3]), "v"(a[4]), "v"(b[4]), "v"(a[5]), "v"(b[5]), "v"(a[6]), "v"(b[6]), "v"(a[7]), "v"(b[7]), "v"(a[8]), "v"(b[8]));
    (void)cc;
  }
};
template <> struct madc<10> {
  static FDG_DEV void run(uint64_t &s, const uint32_t *a, const uint32_t *b) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n" "v_mad_u64_u32 %0, %1, %4, %5, %0\n" "v_mad_u64_u32 %0, %1, %6, %7, %0\n" "v_mad_u64_u32 %0, %1, %8, %9, %0\n" "v_mad_u64_u32 %0, %1, %10, %11, %0\n" "v_mad_u64_u32 %0, %1, %12, %13, %0\n" "v_mad_u64_u32 %0, %1, %14, %15, %0\n" "v_mad_u64_u32 %0, %1, %16, %17, %0\n" "v_mad_u64_u32 %0, %1, %18, %19, %0\n" "v_mad_u64_u32 %0, %1, %20, %21, %0\n"
        : "+v"(s), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(a[1]), "v"(b[1]), "v"(a[2]), "v"(b[2]), "v"(a[3]), "v"(b[3]), "v"(a[4]), "v"(b[4]), "v"(a[5]), "v"(b[5]), "v"(a[6]), "v"(b[6]), "v"(a[7]), "v"(b[7]), "v"(a[8]), "v"(b[8]), "v"(a[9]), "v"(b[9]));
    (void)cc;
  }
};

/* madc0<N>::run(s, a, b): s = a[0] b[0] + ... + a[N-1] b[N-1] -- a column
   chain that starts from zero (column 0 of a product): the first mad takes
   the inline constant 0 as its addend, so no zeroed register pair is
   materialised per product. */
template <int N> struct madc0;
template <> struct madc0<6> {
  static FDG_DEV void run(uint64_t &s, const uint32_t *a, const uint32_t *b) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0\n" "v_mad_u64_u32 %0, %1, %4, %5, %0\n" "v_mad_u64_u32 %0, %1, %6, %7, %0\n" "v_mad_u64_u32 %0, %1, %8, %9, %0\n" "v_mad_u64_u32 %0, %1, %10, %11, %0\n" "v_mad_u64_u32 %0, %1, %12, %13, %0\n"
        : "=&v"(s), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(a[1]), "v"(b[1]), "v"(a[2]), "v"(b[2]), "v"(a[3]), "v"(b[3]), "v"(a[4]), "v"(b[4]), "v"(a[5]), "v"(b[5]));
    (void)cc;
  }
};
template <> struct madc0<10> {
  static FDG_DEV void run(uint64_t &s, const uint32_t *a, const uint32_t *b) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0\n" "v_mad_u64_u32 %0, %1, %4, %5, %0\n" "v_mad_u64_u32 %0, %1, %6, %7, %0\n" "v_mad_u64_u32 %0, %1, %8, %9, %0\n" "v_mad_u64_u32 %0, %1, %10, %11, %0\n" "v_mad_u64_u32 %0, %1, %12, %13, %0\n" "v_mad_u64_u32 %0, %1, %14, %15, %0\n" "v_mad_u64_u32 %0, %1, %16, %17, %0\n" "v_mad_u64_u32 %0, %1, %18, %19, %0\n" "v_mad_u64_u32 %0, %1, %20, %21, %0\n"
        : "=&v"(s), "=&s"(cc) : "v"(a[0]), "v"(b[0]), "v"(a[1]), "v"(b[1]), "v"(a[2]), "v"(b[2]), "v"(a[3]), "v"(b[3]), "v"(a[4]), "v"(b[4]), "v"(a[5]), "v"(b[5]), "v"(a[6]), "v"(b[6]), "v"(a[7]), "v"(b[7]), "v"(a[8]), "v"(b[8]), "v"(a[9]), "v"(b[9]));
    (void)cc;
  }
};

/* Close a feed-forward product: the carry out of column 9 (weight 2^255)
   re-enters limb 0 times 19, and limb 0's excess moves to limb 1
   (carry < 2^39, so limb 1 grows by < 2^17.3). */
FDG_DEV void fe_ff_close(fe &h, uint32_t (&r)[10], uint64_t carry) {
  const uint64_t t = (uint64_t)r[0] + carry * 19u;
  r[0] = (uint32_t)t & ((1u << 26) - 1);
  r[1] += (uint32_t)(t >> 26);
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = r[i];
}

/* h = f * g.  Column k collects f_i g_j with i + j = k (mod 10); a
   product wrapping past 2^255 picks up 19, and an odd-odd limb pair an
   extra 2 (weights 2^ceil(25.5 i)).  f is pre-doubled, g pre-multiplied by
   19, so each term is one v_mad_u64_u32 into a 64-bit column sum. */
FDG_DEV void fe_mul(fe &h, const fe &f, const fe &g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) { g19[i] = 19u * g.v[i]; f2[i] = f.v[i] << 1; }
  uint32_t r[10];
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t s = carry;
    uint32_t ca[10], cb[10];
#pragma unroll
    for (int i = 0; i < 10; i++) {
      int j = k - i;
      const bool wrap = j < 0;
      if (wrap) j += 10;
      const bool dbl = (i & 1) && (j & 1);
      ca[i] = dbl ? f2[i] : f.v[i];
      cb[i] = wrap ? g19[j] : g.v[j];
    }
    if (k == 0) madc0<10>::run(s, ca, cb);
    else madc<10>::run(s, ca, cb);
    const int bits = (k & 1) ? 25 : 26;
    r[k] = (uint32_t)s & ((1u << bits) - 1);
    carry = s >> bits;
  }
  fe_ff_close(h, r, carry);
  FDG_SCHED_FENCE();
}

/* h = 2^SH * f^2 using the symmetric terms once (55 products).  Coefficient
   of f_i f_j (i <= j) in column (i+j) mod 10: (i!=j ? 2 : 1) * (i,j odd ? 2
   : 1) * (i+j >= 10 ? 19 : 1) * 2^SH, applied as (a f_i)(b f_j) with a in
   {1,2,4,8} and b in {1,19} so both factors stay below 2^32 for inputs up to
   A/S (SH = 1 only for R inputs: 8 f_i < 2^30, column sums < 2^62). */
template <int SH>
FDG_DEV void fe_sq_sh(fe &h, const fe &f) {
  uint32_t f2[10], f4[10], f8[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    f2[i] = f.v[i] << 1; f4[i] = f.v[i] << 2; f8[i] = f.v[i] << 3; f19[i] = 19u * f.v[i];
  }
  auto pick = [&](int m, int i) { return m == 0 ? f.v[i] : m == 1 ? f2[i] : m == 2 ? f4[i] : f8[i]; };
  uint32_t r[10];
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t s = carry;
    uint32_t ca[6], cb[6];
    int n = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
      for (int j = i; j < 10; j++) {
        if ((i + j) % 10 != k) continue;
        const int mul2 = (i != j ? 1 : 0) + (((i & 1) && (j & 1)) ? 1 : 0) + SH;
        ca[n] = pick(mul2, i);
        cb[n] = (i + j) >= 10 ? f19[j] : f.v[j];
        n++;
      }
    }
    if (k & 1) madc<5>::run(s, ca, cb);             /* odd columns: 5 symmetric terms, even: 6 */
    else if (k == 0) madc0<6>::run(s, ca, cb);
    else madc<6>::run(s, ca, cb);
    const int bits = (k & 1) ? 25 : 26;
    r[k] = (uint32_t)s & ((1u << bits) - 1);
    carry = s >> bits;
  }
  fe_ff_close(h, r, carry);
  FDG_SCHED_FENCE();
}

FDG_DEV void fe_sq(fe &h, const fe &f) { fe_sq_sh<0>(h, f); }
/* h = 2 f^2 (f <= R) */
FDG_DEV void fe_sq2(fe &h, const fe &f) { fe_sq_sh<1>(h, f); }

FDG_DEV void fe_sqn(fe &h, const fe &f, int n) {
  fe_sq(h, f);
#pragma unroll 1
  for (int i = 1; i < n; i++) fe_sq(h, h);
}

/* Full normalisation to the canonical representative in [0, p). */
FDG_DEV void fe_canon(fe &h) {
  fe_carry(h);
  fe_carry(h);                                   /* value < 2^255 + tiny, limbs normalised except maybe v0 */
  /* q = floor((h + 19) / 2^255) in {0,1} */
  uint32_t q = (h.v[0] + 19u) >> 26;
#pragma unroll
  for (int i = 1; i < 10; i++) q = (h.v[i] + q) >> ((i & 1) ? 25 : 26);
  h.v[0] += 19u * q;
  /* linear carry 0 -> 9, drop 2^255 */
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int w = (i & 1) ? 25 : 26;
    h.v[i + 1] += h.v[i] >> w;
    h.v[i] &= (1u << w) - 1;
  }
  h.v[9] &= (1u << 25) - 1;
}

FDG_DEV bool fe_iszero(const fe &f) {
  fe t = f; fe_canon(t);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) acc |= t.v[i];
  return acc == 0;
}

FDG_DEV uint32_t fe_isodd(const fe &f) { fe t = f; fe_canon(t); return t.v[0] & 1u; }

/* a == b (mod p); a, b <= R (so a + 2p - b stays in 32 bits). */
FDG_DEV bool fe_eq(const fe &a, const fe &b) { fe t; fe_sub(t, a, b); return fe_iszero(t); }

/* Load 32 little-endian bytes (as 8 u32) and drop bit 255: the value is
   NOT reduced mod p (non-canonical y in [p, 2^255) stays as is), exactly
   like the reference's decode (avx512/fd_r43x6_ge.c:195-199). */
FDG_DEV void fe_frombytes(fe &h, const uint32_t (&w)[8]) {
  /* bit positions 0,26,51,77,102,128,153,179,204,230 */
  constexpr int pos[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int p = pos[i], wi = p >> 5, sh = p & 31;
    const int bits = (i & 1) ? 25 : 26;
    uint64_t x = w[wi];
    if (wi + 1 < 8) x |= (uint64_t)w[wi + 1] << 32;
    h.v[i] = (uint32_t)(x >> sh) & ((1u << bits) - 1);
  }
}

/* Canonical little-endian 8 x u32 encoding. */
FDG_DEV void fe_tobytes(uint32_t (&w)[8], const fe &f) {
  fe t = f; fe_canon(t);
  constexpr int pos[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int p = pos[i], wi = p >> 5, sh = p & 31;
    w[wi] |= t.v[i] << sh;
    if (sh && wi + 1 < 8) w[wi + 1] |= t.v[i] >> (32 - sh);
  }
}

/* z^(2^252 - 3) (reference: fd_r43x6.c:98-148 / fd_f25519.c:11-59). */
FDG_DEV void fe_pow22523(fe &out, const fe &z) {
  fe t0, t1, t2;
  fe_sq(t0, z);                           /* 2 */
  fe_sqn(t1, t0, 2);                      /* 8 */
  fe_mul(t1, z, t1);                      /* 9 */
  fe_mul(t0, t0, t1);                     /* 11 */
  fe_sq(t0, t0);                          /* 22 */
  fe_mul(t0, t1, t0);                     /* 2^5 - 1 */
  fe_sqn(t1, t0, 5);   fe_mul(t0, t1, t0);   /* 2^10 - 1 */
  fe_sqn(t1, t0, 10);  fe_mul(t1, t1, t0);   /* 2^20 - 1 */
  fe_sqn(t2, t1, 20);  fe_mul(t1, t2, t1);   /* 2^40 - 1 */
  fe_sqn(t1, t1, 10);  fe_mul(t0, t1, t0);   /* 2^50 - 1 */
  fe_sqn(t1, t0, 50);  fe_mul(t1, t1, t0);   /* 2^100 - 1 */
  fe_sqn(t2, t1, 100); fe_mul(t1, t2, t1);   /* 2^200 - 1 */
  fe_sqn(t1, t1, 50);  fe_mul(t0, t1, t0);   /* 2^250 - 1 */
  fe_sqn(t0, t0, 2);                         /* 2^252 - 4 */
  fe_mul(out, t0, z);                        /* 2^252 - 3 */
}

/* z^(p-2) = 1/z (used only by the B-table initialisation). */
FDG_DEV void fe_invert(fe &out, const fe &z) {
  fe t0, t1, t2, z11;
  fe_sq(t0, z);
  fe_sqn(t1, t0, 2);
  fe_mul(t1, z, t1);
  fe_mul(z11, t0, t1);
  fe_sq(t0, z11);
  fe_mul(t0, t1, t0);
  fe_sqn(t1, t0, 5);   fe_mul(t0, t1, t0);
  fe_sqn(t1, t0, 10);  fe_mul(t1, t1, t0);
  fe_sqn(t2, t1, 20);  fe_mul(t1, t2, t1);
  fe_sqn(t1, t1, 10);  fe_mul(t0, t1, t0);
  fe_sqn(t1, t0, 50);  fe_mul(t1, t1, t0);
  fe_sqn(t2, t1, 100); fe_mul(t1, t2, t1);
  fe_sqn(t1, t1, 50);  fe_mul(t0, t1, t0);
  fe_sqn(t0, t0, 5);
  fe_mul(out, t0, z11);
}

}  // namespace fdgpu
