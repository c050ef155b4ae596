/* fdgpu_lattice.h -- half-size scalars for the verify equation.

   The reference checks [S]B - [k]A == R with a ~253-bit k
   (fd_ed25519_user.c:208-229, fd_curve25519.c:109-153): about 252
   doublings shared by [k]A.  Write N = 8L (the group order is 8L, so every
   decoded point P has [N]P = O).  For any integers (u, v) with
       u = v k  (mod N),   v odd,   0 < |v| < L
   and w = v S mod L:
       [w]B - [u]A - [v]R = [v]([S]B - [k]A - R)
   (B has order L, A and R order dividing 8L), and [v]D = O forces D = O
   because ord(D) divides 8L, an odd v rules out the 2-power part and
   |v| < L rules out L.  So the cofactorless equation -- with any torsion
   component of A or R, exactly the reference's verdict -- is decided by a
   triple scalar multiplication whose variable-base scalars u, v have about
   128 bits: about half the doublings (Antipa et al., "Accelerated
   verification of ECDSA signatures", SAC 2005; Pornin, "Optimized lattice
   basis reduction in dimension 2", 2020, with the modulus N = 8L here so
   the torsion is kept exact rather than cleared).

   (u, v) comes from the extended Euclidean algorithm on (N, k): remainders
   r_i = t_i k (mod N); stopping at the first r_i < 2^128 gives
   |t_i| <= N / r_{i-1} < 2^127.  Of (r_i, t_i), (r_{i-1}, t_{i-1}),
   (r_{i+1}, t_{i+1}), (r_{i-1} - r_i, ...), (r_{i-1} + r_i, ...) the one with
   odd t and the fewest bits is taken (consecutive t are coprime, so an odd
   one exists).  Over 400,000 random k (tests/test_lattice.py's harness):
   99.7% need <= 131 bits (33 radix-16 windows), 5 needed 136-137 bits, none
   more; up to 159 bits (40 windows) run in the verify kernel, and only a
   lane whose Euclid needs a full-precision step with a quotient >= 2^31
   (probability ~2^-30 per step) takes the full-length path
   (fdgpu_kernels.hip, fdgpu_full_kernel).  The Euclid itself runs as
   Lehmer's algorithm (hs_split below).

   Per lane, 32-bit limbs; __host__ __device__ so tests/test_lattice.py can
   check it against Python integers on the CPU. */
#pragma once

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define FDG_HD __host__ __device__ __forceinline__
#else
#define FDG_HD static inline
#endif

namespace fdgpu {

#define HS_MAX_BITS 159u          /* |u|, |v| < 2^159: at most 40 signed radix-16 windows */
#define HS_MAX_ITERS 192u         /* Euclid steps (random k: 43-101; all-ones quotients: ~184) */
#define HS_LIMBS 5u               /* |u|, |v| as 5 x u32 */

/* N = 8L, little-endian u32 limbs */
#define FDGPU_SC_8L { 0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u, 0u, 0u, 0u, 0x80000000u }

FDG_HD uint32_t hs_clz(uint32_t x) { return x ? (uint32_t)__builtin_clz(x) : 32u; }

/* bits of an n-limb unsigned value */
template <int N>
FDG_HD uint32_t hs_bitlen(const uint32_t (&x)[N]) {
  uint32_t bl = 0;
#pragma unroll
  for (int i = 0; i < N; i++) bl = x[i] ? 32u * (uint32_t)(i + 1) - hs_clz(x[i]) : bl;
  return bl;
}

/* bits of |x| for a 6-limb two's complement value */
FDG_HD uint32_t hs_sbitlen(const uint32_t (&x)[6], bool &neg) {
  neg = (x[5] >> 31) != 0;
  uint32_t m[6];
  uint32_t c = 1;
#pragma unroll
  for (int i = 0; i < 6; i++) {                 /* m = neg ? -x : x */
    const uint32_t y = neg ? ~x[i] : x[i];
    const uint64_t s = (uint64_t)y + (neg ? c : 0u);
    m[i] = (uint32_t)s;
    c = (uint32_t)(s >> 32);
  }
  return hs_bitlen<6>(m);
}

/* r = a - q b over 8 limbs; returns the sign of the exact result (true if
   negative, r then holds it mod 2^256) */
FDG_HD bool hs_submul(uint32_t (&r)[8], const uint32_t (&a)[8], uint32_t q, const uint32_t (&b)[8]) {
  uint64_t carry = 0;
  uint32_t borrow = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint64_t p = (uint64_t)q * b[j] + carry;
    carry = p >> 32;
    const uint64_t d = (uint64_t)a[j] - (uint32_t)p - borrow;
    r[j] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
  return (carry + borrow) != 0;
}

/* x += y (8 limbs, mod 2^256) */
FDG_HD void hs_add8(uint32_t (&x)[8], const uint32_t (&y)[8]) {
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint64_t s = (uint64_t)x[j] + y[j] + c;
    x[j] = (uint32_t)s;
    c = (uint32_t)(s >> 32);
  }
}

/* x -= y (8 limbs, mod 2^256) */
FDG_HD void hs_sub8(uint32_t (&x)[8], const uint32_t (&y)[8]) {
  uint32_t bw = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint64_t d = (uint64_t)x[j] - y[j] - bw;
    x[j] = (uint32_t)d;
    bw = (uint32_t)(d >> 63);
  }
}

/* x >= y (8 limbs) */
FDG_HD bool hs_ge8(const uint32_t (&x)[8], const uint32_t (&y)[8]) {
  bool gt = false, eq = true;
#pragma unroll
  for (int i = 7; i >= 0; i--) {
    gt = gt || (eq && x[i] > y[i]);
    eq = eq && x[i] == y[i];
  }
  return gt || eq;
}

/* t = ta - q tb over 6-limb two's complement */
FDG_HD void hs_tsubmul(uint32_t (&t)[6], const uint32_t (&ta)[6], uint32_t q, const uint32_t (&tb)[6]) {
  uint64_t carry = 0;
  uint32_t borrow = 0;
#pragma unroll
  for (int j = 0; j < 6; j++) {
    const uint64_t p = (uint64_t)q * tb[j] + carry;
    carry = p >> 32;
    const uint64_t d = (uint64_t)ta[j] - (uint32_t)p - borrow;
    t[j] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
}

/* t = x + s y (s = +1 / -1) over 6-limb two's complement */
FDG_HD void hs_tadd(uint32_t (&t)[6], const uint32_t (&x)[6], const uint32_t (&y)[6], bool sub) {
  uint32_t c = sub ? 1u : 0u;
#pragma unroll
  for (int j = 0; j < 6; j++) {
    const uint32_t yy = sub ? ~y[j] : y[j];
    const uint64_t s = (uint64_t)x[j] + yy + c;
    t[j] = (uint32_t)s;
    c = (uint32_t)(s >> 32);
  }
}

/* One Euclid quotient of a, b (a > b > 0, a's top limb nonzero after the
   caller's normalisation) from their top 64 bits, exact after correction;
   returns false when the quotient may reach 2^31. */
FDG_HD bool hs_divstep(uint32_t (&r)[8], uint32_t &q, const uint32_t (&a)[8], const uint32_t (&b)[8]) {
  const uint32_t c = hs_clz(a[7]);
  const uint64_t a76 = ((uint64_t)a[7] << 32) | a[6], b76 = ((uint64_t)b[7] << 32) | b[6];
  const uint64_t A = c ? (a76 << c) | (a[5] >> (32u - c)) : a76;
  const uint64_t B = c ? (b76 << c) | (b[5] >> (32u - c)) : b76;
  if ((B >> 32) == 0) return false;                     /* quotient >= 2^31 */
  double qd = (double)A / (double)B;
  q = qd >= 4294967295.0 ? 0xffffffffu : (uint32_t)qd;
  /* |a/b - A/B| < (q + 2) / 2^32: the estimate is within one of floor(a/b) */
  bool neg = hs_submul(r, a, q, b);
#pragma unroll
  for (int it = 0; it < 2; it++) {
    if (neg) {                                          /* too large: r += b */
      uint32_t c0 = 0;
      bool carry_out = false;
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const uint64_t s = (uint64_t)r[j] + b[j] + c0;
        r[j] = (uint32_t)s;
        c0 = (uint32_t)(s >> 32);
      }
      carry_out = c0 != 0;
      neg = !carry_out;                                 /* r was in (-b, 0): the add wraps back to >= 0 */
      q -= 1u;
    }
  }
#pragma unroll
  for (int it = 0; it < 2; it++) {
    if (!neg && hs_ge8(r, b)) { hs_sub8(r, b); q += 1u; }
  }
  return !neg && !hs_ge8(r, b);
}

struct hs_split_t {
  uint32_t u[HS_LIMBS], v[HS_LIMBS];   /* |u|, |v| */
  bool u_neg, v_neg;
  uint32_t bits;                      /* max(bits |u|, bits |v|) */
  bool ok;                            /* false: take the full-length path */
};

/* The candidate (x, t): x >= 0 (8 limbs), t 6-limb two's complement */
FDG_HD void hs_take(hs_split_t &o, const uint32_t (&x)[8], const uint32_t (&t)[6], uint32_t &best, bool valid) {
  bool tneg;
  const uint32_t tb = hs_sbitlen(t, tneg);
  const uint32_t bits = hs_bitlen<8>(x) > tb ? hs_bitlen<8>(x) : tb;
  const bool take = valid && (t[0] & 1u) && bits < best;
  if (!take) return;
  best = bits;
  uint32_t c = 1;
#pragma unroll
  for (int i = 0; i < (int)HS_LIMBS; i++) {
    o.u[i] = x[i];
    const uint32_t y = tneg ? ~t[i] : t[i];
    const uint64_t s = (uint64_t)y + (tneg ? c : 0u);
    o.v[i] = (uint32_t)s;
    c = (uint32_t)(s >> 32);
  }
  o.u_neg = false;
  o.v_neg = tneg;
  o.bits = bits;
}

/* The split from the stopping point of Euclid: ar = r_{i-1} >= 2^128 > br =
   r_i with their cofactors (see the file comment for the candidates). */
FDG_HD void hs_finish(hs_split_t &o, const uint32_t (&ar)[8], const uint32_t (&br)[8], const uint32_t (&ta)[6],
                      const uint32_t (&tb)[6]) {
  o.ok = false;
  o.bits = 0xffffffffu;
  o.u_neg = o.v_neg = false;
#pragma unroll
  for (int i = 0; i < (int)HS_LIMBS; i++) o.u[i] = o.v[i] = 0;
  uint32_t best = HS_MAX_BITS + 1;
  hs_take(o, br, tb, best, true);                                /* (r_i, t_i) */
  hs_take(o, ar, ta, best, true);                                /* (r_{i-1}, t_{i-1}) */
  {                                                              /* (r_{i-1} - r_i, t_{i-1} - t_i) */
    uint32_t x[8], t[6];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = ar[i];
    hs_sub8(x, br);
    hs_tadd(t, ta, tb, true);
    hs_take(o, x, t, best, true);
    uint32_t y[8];                                               /* (r_{i-1} + r_i, t_{i-1} + t_i) */
#pragma unroll
    for (int i = 0; i < 8; i++) y[i] = ar[i];
    hs_add8(y, br);
    hs_tadd(t, ta, tb, false);
    hs_take(o, y, t, best, (ar[7] >> 31) == 0);                  /* no 2^256 wrap */
  }
  {                                                              /* (r_{i+1}, t_{i+1}): one more step */
    bool nz = false;
#pragma unroll
    for (int i = 0; i < 8; i++) nz = nz || br[i] != 0;
    if (nz) {
      /* q = floor(a / b) with b < 2^128: normalise a copy so a's top limb is set */
      uint32_t an[8], bn[8];
#pragma unroll
      for (int i = 0; i < 8; i++) { an[i] = ar[i]; bn[i] = br[i]; }
#pragma unroll 1
      for (int s = 0; s < 7; s++) {
        const bool m = an[7] == 0;
#pragma unroll
        for (int i = 7; i > 0; i--) { an[i] = m ? an[i - 1] : an[i]; bn[i] = m ? bn[i - 1] : bn[i]; }
        an[0] = m ? 0u : an[0];
        bn[0] = m ? 0u : bn[0];
      }
      uint32_t r[8], q = 0;
      if (an[7] != 0 && hs_divstep(r, q, an, bn)) {
        /* r is the normalised remainder; recompute it unshifted: c = a - q b */
        uint32_t c[8], t[6];
        const bool neg = hs_submul(c, ar, q, br);
        hs_tsubmul(t, ta, q, tb);
        hs_take(o, c, t, best, !neg);
      }
    }
  }
  o.ok = best <= HS_MAX_BITS;
}

/* (u, v) for k < L (8 limbs), one full-precision Euclid step per iteration
   -- the definition hs_split (Lehmer) must reproduce; kept for the host
   tests (tests/test_lattice.py). */
FDG_HD void hs_split_euclid(hs_split_t &o, const uint32_t (&k)[8]) {
  constexpr uint32_t NL[8] = FDGPU_SC_8L;
  uint32_t a[8], b[8], ta[6], tb[6];
#pragma unroll
  for (int i = 0; i < 8; i++) { a[i] = NL[i]; b[i] = k[i]; }
#pragma unroll
  for (int i = 0; i < 6; i++) { ta[i] = 0; tb[i] = 0; }
  tb[0] = 1;
  uint32_t sh = 0;                     /* a and b are held shifted left by 32 sh bits */
  bool fail = false, done = false;
#pragma unroll 1
  for (uint32_t it = 0; it < HS_MAX_ITERS; it++) {
    if (!done && !fail) {
      /* normalise: keep a's top limb nonzero (a >= 2^128 while looping, so sh <= 3) */
      const bool s = a[7] == 0;
#pragma unroll
      for (int i = 7; i > 0; i--) { a[i] = s ? a[i - 1] : a[i]; b[i] = s ? b[i - 1] : b[i]; }
      a[0] = s ? 0u : a[0];
      b[0] = s ? 0u : b[0];
      sh += s ? 1u : 0u;
      /* stop at the first remainder below 2^128 (real value b / 2^(32 sh)) */
      uint32_t hi = 0;
#pragma unroll
      for (int j = 4; j < 8; j++) hi |= ((uint32_t)j >= 4u + sh) ? b[j] : 0u;
      done = hi == 0;
      if (!done) {
        uint32_t r[8], q = 0, tr[6];
        if (a[7] == 0 || !hs_divstep(r, q, a, b)) {
          fail = true;
        } else {
          hs_tsubmul(tr, ta, q, tb);
#pragma unroll
          for (int i = 0; i < 8; i++) { a[i] = b[i]; b[i] = r[i]; }
#pragma unroll
          for (int i = 0; i < 6; i++) { ta[i] = tb[i]; tb[i] = tr[i]; }
        }
      }
    }
#if defined(__HIP_DEVICE_COMPILE__)
    if (__all(done || fail)) break;
#else
    if (done || fail) break;
#endif
  }
  o.ok = false;
  o.bits = 0xffffffffu;
  o.u_neg = o.v_neg = false;
#pragma unroll
  for (int i = 0; i < (int)HS_LIMBS; i++) o.u[i] = o.v[i] = 0;
  if (fail || !done) return;
  /* un-shift to real values */
  uint32_t ar[8], br[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t xa = 0, xb = 0;
#pragma unroll
    for (uint32_t s = 0; s <= 4; s++) {
      const bool in = (uint32_t)i + s < 8u;
      xa = sh == s ? (in ? a[(i + s) & 7] : 0u) : xa;
      xb = sh == s ? (in ? b[(i + s) & 7] : 0u) : xb;
    }
    ar[i] = xa;
    br[i] = xb;
  }
  hs_finish(o, ar, br, ta, tb);
}

/* ---- Lehmer's algorithm (Knuth, TAOCP vol. 2, 4.5.2, Algorithm L) ----
   The Euclid steps are simulated on the leading 52 bits of a and b in
   doubles (exact: every value stays below 2^53), collecting the 2x2
   cofactor matrix; a quotient is taken only when both bracketing ratios
   (U + A)/(V + C) and (U + B)/(V + D) agree on it, so the simulated steps
   are exactly Euclid's.  The matrix is then applied to the full values
   (about 26 bits of reduction per application instead of ~1.2 per
   full-width step).  The stop rule is Euclid's too: a step is taken inside
   the simulation only when its remainder is known to be >= 2^128 or known
   to be < 2^128 (then it is the last); an undecided step, or a first step
   the brackets cannot settle, is taken at full precision.  So hs_split
   ends at the same (r_{i-1}, r_i) as hs_split_euclid and returns the same
   split (tests/test_lattice.py checks this). */
#define HS_MAX_OUTER 200u     /* matrix applications + full steps (random k: ~6-10) */
#define HS_MAX_INNER 48u      /* simulated steps per application (cofactors < 2^31) */

/* 1/y to ~2^-52 relative: the hardware reciprocal (v_rcp_f64) and one
   Newton step on the device, a division on the host */
FDG_HD double hs_rcp(double y) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double r = __builtin_amdgcn_rcp(y);
  return fma(r, fma(-y, r, 1.0), r);
#else
  return 1.0 / y;
#endif
}

/* floor(x / y) for integers 0 <= x < 2^53, 0 < y < 2^53 held in doubles.
   The estimate floor(x * (1/y)) is within one of the floor while the
   quotient is below ~2^50 (every quotient the Lehmer simulation can take
   is below 2^31: a larger one breaks it on the cofactor bound), and the
   remainder x - q y is exact (an integer of magnitude < 2y < 2^54 computed
   by one fma; its sign and its comparison with y are exact even when it
   rounds), so one correction step gives the floor. */
FDG_HD double hs_fdivf(double x, double y) {
  const double q = floor(x * hs_rcp(y));
  const double r = fma(-q, y, x);
  return r < 0.0 ? q - 1.0 : (r >= y ? q + 1.0 : q);
}

/* q == floor(x / y) for integers 0 <= x < 2^53, 0 < y < 2^53: the remainder
   x - q y lies in [0, y) (one fma, exact as above) */
FDG_HD bool hs_isquot(double q, double x, double y) {
  const double r = fma(-q, y, x);
  return r >= 0.0 && r < y;
}

/* (x >> s) for an 8-limb x < 2^(s + 64), s < 256 (selects, no dynamic
   register indexing) */
FDG_HD uint64_t hs_window(const uint32_t (&x)[8], uint32_t s) {
  const uint32_t w = s >> 5, o = s & 31u;
  uint32_t l0 = 0, l1 = 0, l2 = 0;
#pragma unroll
  for (uint32_t i = 0; i < 8; i++) {
    l0 = i == w ? x[i] : l0;
    l1 = i == w + 1u ? x[i] : l1;
    l2 = i == w + 2u ? x[i] : l2;
  }
  const uint64_t lo = ((uint64_t)l1 << 32) | l0;
  return o ? (lo >> o) | ((uint64_t)l2 << (64u - o)) : lo;
}

/* o = cx x + cy y over N limbs (mod 2^(32N)), cx and cy of opposite signs
   (or one of them 0) with magnitudes < 2^31: o = +-(|cx| x - |cy| y).  For
   remainders the true value is in [0, 2^256); for the two's complement
   cofactors it fits N limbs. */
template <int N>
FDG_HD void hs_lin(uint32_t (&o)[N], const uint32_t (&x)[N], double cx, const uint32_t (&y)[N], double cy) {
  const bool flip = cx < 0.0 || (cx == 0.0 && cy > 0.0);
  const uint32_t mx = (uint32_t)fabs(cx), my = (uint32_t)fabs(cy);
  uint64_t cp = 0, cq = 0;
  uint32_t bw = 0;
#pragma unroll
  for (int j = 0; j < N; j++) {
    const uint64_t p = (uint64_t)mx * x[j] + cp, q = (uint64_t)my * y[j] + cq;
    cp = p >> 32;
    cq = q >> 32;
    const uint32_t pos = flip ? (uint32_t)q : (uint32_t)p, neg = flip ? (uint32_t)p : (uint32_t)q;
    const uint64_t d = (uint64_t)pos - neg - bw;
    o[j] = (uint32_t)d;
    bw = (uint32_t)(d >> 63);
  }
}

/* One full-precision Euclid step (a, b, ta, tb) <- (b, a - q b, tb, ta - q tb);
   false when the quotient may reach 2^31 (the lane takes the full path). */
FDG_HD bool hs_fullstep(uint32_t (&a)[8], uint32_t (&b)[8], uint32_t (&ta)[6], uint32_t (&tb)[6]) {
  uint32_t an[8], bn[8];
#pragma unroll
  for (int i = 0; i < 8; i++) { an[i] = a[i]; bn[i] = b[i]; }
#pragma unroll 1
  for (int s = 0; s < 7; s++) {                 /* normalise copies: a's top limb set */
    const bool m = an[7] == 0;
#pragma unroll
    for (int i = 7; i > 0; i--) { an[i] = m ? an[i - 1] : an[i]; bn[i] = m ? bn[i - 1] : bn[i]; }
    an[0] = m ? 0u : an[0];
    bn[0] = m ? 0u : bn[0];
  }
  uint32_t r[8], q = 0;
  if (an[7] == 0 || !hs_divstep(r, q, an, bn)) return false;
  uint32_t c[8], t[6];
  (void)hs_submul(c, a, q, b);                  /* q is exact: c = a mod b >= 0 */
  hs_tsubmul(t, ta, q, tb);
#pragma unroll
  for (int i = 0; i < 8; i++) { a[i] = b[i]; b[i] = c[i]; }
#pragma unroll
  for (int i = 0; i < 6; i++) { ta[i] = tb[i]; tb[i] = t[i]; }
  return true;
}

/* (u, v) for k < L (8 limbs) -- see the file comment. */
FDG_HD void hs_split(hs_split_t &o, const uint32_t (&k)[8]) {
  constexpr uint32_t NL[8] = FDGPU_SC_8L;
  uint32_t a[8], b[8], ta[6], tb[6];
#pragma unroll
  for (int i = 0; i < 8; i++) { a[i] = NL[i]; b[i] = k[i]; }
#pragma unroll
  for (int i = 0; i < 6; i++) { ta[i] = 0; tb[i] = 0; }
  tb[0] = 1;
  bool fail = false, done = false;
#pragma unroll 1
  for (uint32_t it = 0; it < HS_MAX_OUTER; it++) {
    if (!done && !fail) {
      done = (b[4] | b[5] | b[6] | b[7]) == 0;   /* r_i < 2^128 (a = r_{i-1} >= 2^128) */
      if (!done) {
        const uint32_t s = hs_bitlen<8>(a) - 52u;   /* a >= 2^128: s >= 77 */
        double U = (double)hs_window(a, s), V = (double)hs_window(b, s);
        const double T = ldexp(1.0, 128 - (int)s);   /* 2^128 in units of 2^s */
        double A = 1.0, B = 0.0, C = 0.0, D = 1.0;
#pragma unroll 1
        for (uint32_t j = 0; j < HS_MAX_INNER; j++) {
          if (V + C <= 0.0 || V + D <= 0.0) break;
          const double q = hs_fdivf(U + A, V + C);
          if (!hs_isquot(q, U + B, V + D)) break;     /* both brackets agree on q */
          const double Vn = fma(-q, V, U), Cn = fma(-q, C, A), Dn = fma(-q, D, B);
          if (fmax(fabs(Cn), fabs(Dn)) >= 2147483648.0) break;
          /* the true remainder / 2^s lies in (Vn + min(Cn, Dn), Vn + max(Cn, Dn)) */
          const double lo = Vn + fmin(Cn, Dn), hi = Vn + fmax(Cn, Dn);
          if (hi > T && lo < T) break;            /* undecided: take it at full precision */
          U = V; V = Vn; A = C; C = Cn; B = D; D = Dn;
          if (hi <= T) break;                     /* the first remainder below 2^128: stop */
        }
        if (B == 0.0) {
          fail = !hs_fullstep(a, b, ta, tb);
        } else {
          uint32_t a2[8], b2[8], ta2[6], tb2[6];
          hs_lin<8>(a2, a, A, b, B);
          hs_lin<8>(b2, a, C, b, D);
          hs_lin<6>(ta2, ta, A, tb, B);
          hs_lin<6>(tb2, ta, C, tb, D);
#pragma unroll
          for (int i = 0; i < 8; i++) { a[i] = a2[i]; b[i] = b2[i]; }
#pragma unroll
          for (int i = 0; i < 6; i++) { ta[i] = ta2[i]; tb[i] = tb2[i]; }
        }
      }
    }
#if defined(__HIP_DEVICE_COMPILE__)
    if (__all(done || fail)) break;
#else
    if (done || fail) break;
#endif
  }
  if (fail || !done) {
    o.ok = false;
    o.bits = 0xffffffffu;
    o.u_neg = o.v_neg = false;
#pragma unroll
    for (int i = 0; i < (int)HS_LIMBS; i++) o.u[i] = o.v[i] = 0;
    return;
  }
  hs_finish(o, a, b, ta, tb);
}

}  // namespace fdgpu
