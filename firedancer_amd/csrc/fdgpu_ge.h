/* fdgpu_ge.h -- Ed25519 group arithmetic (twisted Edwards, a = -1) per lane.

   Extended coordinates (Hisil-Wong-Carter-Dawson 2008), the same group law
   as the reference's avx512/fd_r43x6_ge.h:119-236 (ADD, ADD_TABLE, DBL);
   any exact formula yields the same group element, which is all the
   verify contract observes.

     p2    (X:Y:Z)                     x = X/Z, y = Y/Z
     p3    (X:Y:Z:T)                   + T = XY/Z
     p1p1  ((X:Z),(Y:T))               x = X/Z, y = Y/T   (completed)
     cached (Y+X, Y-X, 2Z, 2dT)        table entries for the variable base
     niels  (y+x, y-x, 2dxy)           affine table entries for B
   Operand bounds (see fdgpu_fe.h) are annotated at each product. */
#pragma once

#include "fdgpu_fe.h"

namespace fdgpu {

struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };
struct ge_cached { fe YpX, YmX, Z2, T2d; };
struct ge_niels { fe ypx, ymx, xy2d; };

FDG_DEV void ge_p2_0(ge_p2 &h) { fe_0(h.X); fe_1(h.Y); fe_1(h.Z); }
FDG_DEV void ge_p3_0(ge_p3 &h) { fe_0(h.X); fe_1(h.Y); fe_1(h.Z); fe_0(h.T); }
FDG_DEV void ge_cached_0(ge_cached &h) { fe_1(h.YpX); fe_1(h.YmX); fe_0(h.Z2); h.Z2.v[0] = 2; fe_0(h.T2d); }

/* p1p1 -> p2: 3M.  X' (S4|S) first operand, T' (R|S) second; Z' (S|A|2^27.6)
   first x Y' (A) second.  Operand roles are fixed per coordinate (X', Z'
   always first, T', Y' always second) so the pre-scaled operands fe_mul
   derives (2f on odd limbs of the first, 19g of the second) are computed
   once per coordinate and shared by the products that reuse it (and by the
   T = X'Y' product the chain adds for a p3). */
FDG_DEV void ge_p1p1_to_p2(ge_p2 &r, const ge_p1p1 &p) {
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Z, p.Y);
  fe_mul(r.Z, p.Z, p.T);
}
/* p1p1 -> p3: 4M (roles as in ge_p1p1_to_p2). */
FDG_DEV void ge_p1p1_to_p3(ge_p3 &r, const ge_p1p1 &p) {
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Z, p.Y);
  fe_mul(r.Z, p.Z, p.T);
  fe_mul(r.T, p.X, p.Y);
}

/* 2P from p2 (R coords): 4S.
     XX = X^2, YY = Y^2, B = 2 Z^2 (A), AA = (X+Y)^2
     Y' = YY + XX (A), Z' = YY - XX (S), X' = AA - Y' (S4), T' = B - Z' -> carried to R.
   Downstream products: X'T' (S4 x R), Y'Z' (A x S), Z'T' (S x R), X'Y' (S4 x A).
   Written in the order that keeps the fewest field elements live. */
FDG_DEV void ge_dbl(ge_p1p1 &r, const ge_p2 &p) {
  fe s;
  fe_sq(r.X, p.X);                 /* XX */
  fe_sq(r.Z, p.Y);                 /* YY */
  fe_add(r.Y, r.Z, r.X);           /* Y' = YY + XX */
  fe_sub(r.Z, r.Z, r.X);           /* Z' = YY - XX */
  fe_add(s, p.X, p.Y);
  fe_sq(r.X, s);                   /* AA */
  fe_sub4(r.X, r.X, r.Y);          /* X' = AA - Y' */
  fe_sq2(r.T, p.Z);                /* B = 2 Z^2 (R) */
  fe_sub4(r.T, r.T, r.Z);          /* T' = B - Z' */
  fe_carry_par(r.T);
}

FDG_DEV void fe_cswap(fe &a, fe &b, bool c) {
#pragma unroll
  for (int i = 0; i < 10; i++) { const uint32_t x = a.v[i], y = b.v[i]; a.v[i] = c ? y : x; b.v[i] = c ? x : y; }
}
/* a = c ? 2p - a : a  (a <= R; output <= 2^27) */
FDG_DEV void fe_cneg(fe &a, bool c) {
  constexpr uint32_t P2[10] = FDGPU_FE_2P;
#pragma unroll
  for (int i = 0; i < 10; i++) a.v[i] = c ? P2[i] - a.v[i] : a.v[i];
}

/* P + Q with Q cached (entries stored R): 4M.  q is consumed (modified).
   T1 R x T2d (R, or <= 2^27 when negated); Z1 R x Z2 R;
   (Y1+X1) A x YpX R; (Y1-X1) S x YmX R.
   Outputs X' = A-B (S), Y' = A+B (A), Z' = D+C (A), T' = D-C (S).
   neg selects P - Q (swap YpX/YmX, negate T2d). */
FDG_DEV void ge_add_cached(ge_p1p1 &r, const ge_p3 &p, ge_cached q, bool neg) {
  fe t;
  fe_cswap(q.YpX, q.YmX, neg);
  fe_cneg(q.T2d, neg);
  fe_mul(r.Z, p.T, q.T2d);         /* C */
  fe_mul(r.T, p.Z, q.Z2);          /* D */
  fe_add(t, p.Y, p.X);
  fe_mul(r.X, t, q.YpX);           /* A */
  fe_sub(t, p.Y, p.X);
  fe_mul(r.Y, t, q.YmX);           /* B */
  fe_add(t, r.T, r.Z);             /* D + C */
  fe_sub(r.T, r.T, r.Z);           /* D - C */
  r.Z = t;
  fe_add(t, r.X, r.Y);             /* A + B */
  fe_sub(r.X, r.X, r.Y);           /* A - B */
  r.Y = t;
}

/* P + Q with Q affine niels (Z2 = 1): 3M.  q is consumed.  D = 2 Z1 (A);
   Z' = D + C (<= 2^27.6, second operand only), T' = D - C carried to R. */
FDG_DEV void ge_add_niels(ge_p1p1 &r, const ge_p3 &p, ge_niels q, bool neg) {
  fe t;
  fe_cswap(q.ypx, q.ymx, neg);
  fe_cneg(q.xy2d, neg);
  fe_mul(r.Z, p.T, q.xy2d);        /* C */
  fe_add(r.T, p.Z, p.Z);           /* D */
  fe_add(t, p.Y, p.X);
  fe_mul(r.X, t, q.ypx);           /* A */
  fe_sub(t, p.Y, p.X);
  fe_mul(r.Y, t, q.ymx);           /* B */
  fe_add(t, r.T, r.Z);             /* D + C */
  fe_sub(r.T, r.T, r.Z);           /* D - C */
  fe_carry(r.T);
  r.Z = t;
  fe_add(t, r.X, r.Y);
  fe_sub(r.X, r.X, r.Y);
  r.Y = t;
}

/* Table-streaming variants: each table coordinate is read right before the
   product that consumes it (the scheduling fence after every product keeps
   the loads from being hoisted), so at most one coordinate of the entry is
   live.  `ld(i, w)` returns word w (0..9) of coordinate i of the entry.
   Coordinate order in the entry: 0 = Y+X, 1 = Y-X, 2 = 2Z (cached only),
   last = 2dT.  neg selects P - Q by reading Y+X/Y-X swapped and negating 2dT. */
template <class LD>
FDG_DEV void ld_fe(fe &h, const LD &ld, int coord) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = ld(coord, i);
}

template <class LD>
FDG_DEV void ge_add_cached_ld(ge_p1p1 &r, const ge_p3 &p, const LD &ld, bool neg) {
  fe t, q;
  ld_fe(q, ld, 3); fe_cneg(q, neg);
  fe_mul(r.Z, p.T, q);             /* C = T1 2dT2 */
  ld_fe(q, ld, 2);
  fe_mul(r.T, p.Z, q);             /* D = Z1 2Z2 */
  ld_fe(q, ld, neg ? 1 : 0);
  fe_add(t, p.Y, p.X);
  fe_mul(r.X, t, q);               /* A */
  ld_fe(q, ld, neg ? 0 : 1);
  fe_sub(t, p.Y, p.X);
  fe_mul(r.Y, t, q);               /* B */
  fe_add(t, r.T, r.Z);
  fe_sub(r.T, r.T, r.Z);
  r.Z = t;
  fe_add(t, r.X, r.Y);
  fe_sub(r.X, r.X, r.Y);
  r.Y = t;
}

template <class LD>
FDG_DEV void ge_add_niels_ld(ge_p1p1 &r, const ge_p3 &p, const LD &ld, bool neg) {
  fe t, q;
  ld_fe(q, ld, 2); fe_cneg(q, neg);
  fe_mul(r.Z, p.T, q);             /* C = T1 2dxy */
  fe_add(r.T, p.Z, p.Z);           /* D = 2 Z1 */
  ld_fe(q, ld, neg ? 1 : 0);
  fe_add(t, p.Y, p.X);
  fe_mul(r.X, t, q);               /* A */
  ld_fe(q, ld, neg ? 0 : 1);
  fe_sub(t, p.Y, p.X);
  fe_mul(r.Y, t, q);               /* B */
  fe_add(t, r.T, r.Z);
  fe_sub(r.T, r.T, r.Z);
  fe_carry_par(r.T);
  r.Z = t;
  fe_add(t, r.X, r.Y);
  fe_sub(r.X, r.X, r.Y);
  r.Y = t;
}

/* ge_add_cached_ld over an entry already in registers (q: the 40 words of a
   cached entry, coordinate order as above).  The Y+X / Y-X swap for neg is a
   per-word select, so no register array is indexed dynamically. */
FDG_DEV void ge_add_cached_regs(ge_p1p1 &r, const ge_p3 &p, const uint32_t (&q)[40], bool neg) {
  fe t, c;
#pragma unroll
  for (int i = 0; i < 10; i++) c.v[i] = q[30 + i];
  fe_cneg(c, neg);
  fe_mul(r.Z, p.T, c);             /* C = T1 2dT2 */
#pragma unroll
  for (int i = 0; i < 10; i++) c.v[i] = q[20 + i];
  fe_mul(r.T, p.Z, c);             /* D = Z1 2Z2 */
#pragma unroll
  for (int i = 0; i < 10; i++) c.v[i] = neg ? q[10 + i] : q[i];
  fe_add(t, p.Y, p.X);
  fe_mul(r.X, t, c);               /* A */
#pragma unroll
  for (int i = 0; i < 10; i++) c.v[i] = neg ? q[i] : q[10 + i];
  fe_sub(t, p.Y, p.X);
  fe_mul(r.Y, t, c);               /* B */
  fe_add(t, r.T, r.Z);
  fe_sub(r.T, r.T, r.Z);
  r.Z = t;
  fe_add(t, r.X, r.Y);
  fe_sub(r.X, r.X, r.Y);
  r.Y = t;
}

/* ge_add_cached_regs with the Y+X / Y-X swap for neg already applied by the
   caller (q[0..9] multiplies Y1+X1, q[10..19] Y1-X1); neg still negates 2dT. */
FDG_DEV void ge_add_cached_regs_swapped(ge_p1p1 &r, const ge_p3 &p, const uint32_t (&q)[40], bool neg) {
  fe t, c;
#pragma unroll
  for (int i = 0; i < 10; i++) c.v[i] = q[30 + i];
  fe_cneg(c, neg);
  fe_mul(r.Z, p.T, c);             /* C = T1 2dT2 */
#pragma unroll
  for (int i = 0; i < 10; i++) c.v[i] = q[20 + i];
  fe_mul(r.T, p.Z, c);             /* D = Z1 2Z2 */
#pragma unroll
  for (int i = 0; i < 10; i++) c.v[i] = q[i];
  fe_add(t, p.Y, p.X);
  fe_mul(r.X, t, c);               /* A */
#pragma unroll
  for (int i = 0; i < 10; i++) c.v[i] = q[10 + i];
  fe_sub(t, p.Y, p.X);
  fe_mul(r.Y, t, c);               /* B */
  fe_add(t, r.T, r.Z);
  fe_sub(r.T, r.T, r.Z);
  r.Z = t;
  fe_add(t, r.X, r.Y);
  fe_sub(r.X, r.X, r.Y);
  r.Y = t;
}

/* A cached entry in registers (Y+X, Y-X, 2Z, 2dT) as a p2 point:
   (Y+X) - (Y-X) = 2X and (Y+X) + (Y-X) = 2Y over 2Z are the same projective
   point.  neg gives -P (Y+X and Y-X swapped).  X, Y carried to R; Z = the
   entry's 2Z (R). */
FDG_DEV void ge_cached_regs_to_p2(ge_p2 &r, const uint32_t (&q)[40], bool neg) {
  fe a, b;
#pragma unroll
  for (int i = 0; i < 10; i++) { a.v[i] = neg ? q[10 + i] : q[i]; b.v[i] = neg ? q[i] : q[10 + i]; }
  fe_sub(r.X, a, b); fe_carry(r.X);
  fe_add(r.Y, a, b); fe_carry(r.Y);
#pragma unroll
  for (int i = 0; i < 10; i++) r.Z.v[i] = q[20 + i];
}

/* An affine niels entry in registers (y+x, y-x, 2dxy) as a p3 point:
   X' = (y+x) - (y-x) = 2x, Y' = 2y, and (2X', 2Y', 4, X'Y') = 4 (x, y, 1, xy).
   neg gives -P.  1M; X, Y carried to R. */
FDG_DEV void ge_niels_regs_to_p3(ge_p3 &r, const uint32_t (&q)[32], bool neg) {
  fe a, b, x2, y2;
#pragma unroll
  for (int i = 0; i < 10; i++) { a.v[i] = neg ? q[10 + i] : q[i]; b.v[i] = neg ? q[i] : q[10 + i]; }
  fe_sub(x2, a, b); fe_carry(x2);
  fe_add(y2, a, b); fe_carry(y2);
  fe_mul(r.T, x2, y2);
  fe_add(r.X, x2, x2); fe_carry(r.X);
  fe_add(r.Y, y2, y2); fe_carry(r.Y);
  fe_0(r.Z); r.Z.v[0] = 4;
}

/* P + Q with Q an affine niels entry in registers (q[0..9] = y+x,
   q[10..19] = y-x, q[20..29] = 2dxy, canonical): 3M.  neg selects P - Q. */
FDG_DEV void ge_add_niels_regs(ge_p1p1 &r, const ge_p3 &p, const uint32_t (&q)[32], bool neg) {
  fe t, c;
#pragma unroll
  for (int i = 0; i < 10; i++) c.v[i] = q[20 + i];
  fe_cneg(c, neg);
  fe_mul(r.Z, p.T, c);             /* C = T1 2dxy */
  fe_add(r.T, p.Z, p.Z);           /* D = 2 Z1 */
#pragma unroll
  for (int i = 0; i < 10; i++) c.v[i] = neg ? q[10 + i] : q[i];
  fe_add(t, p.Y, p.X);
  fe_mul(r.X, t, c);               /* A */
#pragma unroll
  for (int i = 0; i < 10; i++) c.v[i] = neg ? q[i] : q[10 + i];
  fe_sub(t, p.Y, p.X);
  fe_mul(r.Y, t, c);               /* B */
  fe_add(t, r.T, r.Z);
  fe_sub(r.T, r.T, r.Z);
  fe_carry_par(r.T);
  r.Z = t;
  fe_add(t, r.X, r.Y);
  fe_sub(r.X, r.X, r.Y);
  r.Y = t;
}

FDG_DEV void ge_p3_to_cached(ge_cached &r, const ge_p3 &p) {
  constexpr uint32_t D2[10] = FDGPU_FE_D2;
  fe d2; fe_set(d2, D2);
  fe_add(r.YpX, p.Y, p.X); fe_carry(r.YpX);
  fe_sub(r.YmX, p.Y, p.X); fe_carry(r.YmX);
  fe_add(r.Z2, p.Z, p.Z);  fe_carry(r.Z2);
  fe_mul(r.T2d, p.T, d2);
}

FDG_DEV void ge_p3_to_p2(ge_p2 &r, const ge_p3 &p) { r.X = p.X; r.Y = p.Y; r.Z = p.Z; }

/* -P (X and T negated), outputs carried to R. */
FDG_DEV void ge_p3_neg(ge_p3 &r, const ge_p3 &p) {
  fe_neg(r.X, p.X); fe_carry(r.X);
  r.Y = p.Y; r.Z = p.Z;
  fe_neg(r.T, p.T); fe_carry(r.T);
}

/* Point decoding with the AVX-512 backend's rules
   (avx512/fd_r43x6_ge.c:163-254):
     y = enc & (2^255 - 1) (non-canonical accepted), sign = bit 255
     u = y^2 - 1, v = d y^2 + 1, x = u v^3 (u v^7)^((p-5)/8)
     fail if v x^2 != +-u; x *= sqrt(-1) if v x^2 == -u
     fail if x == 0 and sign == 1 (ref_map: accepted); negate x if parity != sign.
   Returns true on success; P = (x, y, 1, xy) with R-bound coordinates. */
FDG_DEV bool ge_decode(ge_p3 &P, const uint32_t (&enc)[8], bool ref_map) {
  constexpr uint32_t DD[10] = FDGPU_FE_D, SQ[10] = FDGPU_FE_SQRTM1;
  fe d, sqrtm1, one;
  fe_set(d, DD); fe_set(sqrtm1, SQ); fe_1(one);
  const uint32_t sign = enc[7] >> 31;
  fe y, ysq, u, v, v2, v3, v4, uv3, uv7, t0, x, x2, vx2, t1, t2;
  fe_frombytes(y, enc);
  fe_sq(ysq, y);
  fe_sub(u, ysq, one);                    /* S */
  fe_mul(v, d, ysq); fe_add(v, v, one);   /* R + 1 */
  fe_sq(v2, v);
  fe_sq(v4, v2);
  fe_mul(v3, v, v2);
  fe_mul(uv3, u, v3);
  fe_mul(uv7, uv3, v4);
  fe_pow22523(t0, uv7);
  fe_mul(x, uv3, t0);
  fe_sq(x2, x);
  fe_mul(vx2, v, x2);
  fe_carry(u);                            /* u <= R for the subtractions below */
  fe_sub(t1, vx2, u);
  fe_add(t2, vx2, u);
  const bool t1nz = !fe_iszero(t1), t2nz = !fe_iszero(t2);
  bool ok = !(t1nz && t2nz);
  fe xs; fe_mul(xs, x, sqrtm1);
  fe_cmov(x, xs, x, t1nz);
  fe xc = x; fe_canon(xc);
  uint32_t xnz = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) xnz |= xc.v[i];
  if (!ref_map && xnz == 0 && sign) ok = false;
  fe nx; fe_neg(nx, xc); fe_carry(nx);
  fe_cmov(x, nx, xc, (xc.v[0] & 1u) != sign);
  P.X = x; P.Y = y; fe_1(P.Z); fe_mul(P.T, x, y);
  return ok;
}

/* [8]P == O for an affine point (Z = 1): x == 0, y == 0, y == y0 or y == y1
   (fd_curve25519.h:84-114), evaluated on canonical residues. */
FDG_DEV bool ge_is_small_order_affine(const ge_p3 &P) {
  constexpr uint32_t Y0[10] = FDGPU_FE_Y0, Y1[10] = FDGPU_FE_Y1;
  fe y0, y1; fe_set(y0, Y0); fe_set(y1, Y1);
  fe yc = P.Y; fe_canon(yc);
  bool yz = true, e0 = true, e1 = true;
#pragma unroll
  for (int i = 0; i < 10; i++) { yz &= yc.v[i] == 0; e0 &= yc.v[i] == y0.v[i]; e1 &= yc.v[i] == y1.v[i]; }
  return fe_iszero(P.X) || yz || e0 || e1;
}

}  // namespace fdgpu
