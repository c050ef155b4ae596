/* fdgpu_sc.h -- scalars mod L on gfx950 (32-bit limbs).

   sc_validate: S < L, i.e. fd_curve25519_scalar_validate's S <= L-1
     (fd_curve25519_scalar.h:57-73).
   sc_reduce512: k = x mod L for the 512-bit hash (the reference's
     fd_curve25519_scalar_reduce, fd_curve25519_scalar.c:4-110), here as
     Barrett reduction (HAC 14.42, b = 2^32, k = 8, mu = floor(2^512/L)).
   Recoding into fixed signed windows replaces the reference's wNAF
     (fd_curve25519_scalar.c:277-360): every lane of a wave then adds at the
     same loop positions (no divergence), and the represented integer is
     unchanged, so the resulting point is identical. */
#pragma once

#include "fdgpu_fe.h"

namespace fdgpu {

FDG_DEV bool sc_lt_L(const uint32_t (&s)[8]) {
  constexpr uint32_t L[8] = FDGPU_SC_L;
  bool lt = false, eq = true;
#pragma unroll
  for (int i = 7; i >= 0; i--) {
    lt = lt || (eq && s[i] < L[i]);
    eq = eq && s[i] == L[i];
  }
  return lt;
}

FDG_DEV void sc_reduce512(uint32_t (&r)[8], const uint32_t (&x)[16]) {
  constexpr uint32_t MU[9] = FDGPU_SC_MU;
  constexpr uint32_t L[8] = FDGPU_SC_L;
  /* q1 = x >> 224 (9 words); q3 = (q1 * mu) >> 288 (9 words) */
  uint32_t q1[9];
#pragma unroll
  for (int i = 0; i < 9; i++) q1[i] = x[7 + i];
  uint32_t q2[18];
#pragma unroll
  for (int i = 0; i < 18; i++) q2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) {
      const uint64_t t = (uint64_t)q1[i] * MU[j] + q2[i + j] + c;
      q2[i + j] = (uint32_t)t; c = t >> 32;
    }
    q2[i + 9] = (uint32_t)c;
  }
  /* r2 = (q3 * L) mod b^9 */
  uint32_t r2[9];
#pragma unroll
  for (int i = 0; i < 9; i++) r2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (i + j >= 9) break;
      const uint64_t t = (uint64_t)q2[9 + i] * L[j] + r2[i + j] + c;
      r2[i + j] = (uint32_t)t; c = t >> 32;
    }
    if (i + 8 < 9) r2[i + 8] += (uint32_t)c;
  }
  /* r = (x mod b^9) - r2 mod b^9 */
  uint32_t rr[9];
  uint64_t bw = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint64_t t = (uint64_t)x[i] - r2[i] - bw;
    rr[i] = (uint32_t)t; bw = (t >> 63) & 1;
  }
  /* at most two conditional subtractions of L */
#pragma unroll
  for (int it = 0; it < 2; it++) {
    bool ge = rr[8] != 0, eq = rr[8] == 0;
#pragma unroll
    for (int i = 7; i >= 0; i--) {
      ge = ge || (eq && rr[i] > L[i]);
      eq = eq && rr[i] == L[i];
    }
    ge = ge || eq;
    uint64_t b2 = 0;
    uint32_t s[9];
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const uint64_t t = (uint64_t)rr[i] - (i < 8 ? L[i] : 0u) - b2;
      s[i] = (uint32_t)t; b2 = (t >> 63) & 1;
    }
#pragma unroll
    for (int i = 0; i < 9; i++) rr[i] = ge ? s[i] : rr[i];
  }
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = rr[i];
}

/* Signed radix-16 digits of k (< 2^253): 64 digits in [-8, 7], packed as
   4-bit two's complement nibbles into 8 words, digit i at bits 4(i%8) of word i/8. */
FDG_DEV void sc_recode16(uint32_t (&out)[8], const uint32_t (&k)[8]) {
  uint32_t carry = 0;
#pragma unroll
  for (int w = 0; w < 8; w++) {
    uint32_t o = 0;
#pragma unroll
    for (int n = 0; n < 8; n++) {
      uint32_t e = ((k[w] >> (4 * n)) & 15u) + carry;
      carry = e >= 8u;
      e = (e - (carry << 4)) & 15u;   /* two's complement nibble */
      o |= e << (4 * n);
    }
    out[w] = o;
  }
}

/* Signed radix-2^W digits of S for the fixed-base comb (W = FDGPU_BCOMB_BITS):
   NDIG digits d_i in [-2^(W-1), 2^(W-1)), S = sum d_i 2^(W i), packed in
   COMB_SLOT(W)-bit two's complement slots (two int16 per word for W <= 16,
   one per word above; digit 0 in the low slot of word 0).  Needs
   S < 2^(W NDIG - 1) (callers pass S < L or 0). */
#define COMB_SLOT(W) ((W) <= 16 ? 16 : 32)
#define COMB_WORDS(W, NDIG) (((NDIG) * COMB_SLOT(W) + 31) / 32)
template <int W, int NDIG>
FDG_DEV void sc_recode_comb(uint32_t (&out)[COMB_WORDS(W, NDIG)], const uint32_t (&s)[8]) {
  constexpr int SLOT = COMB_SLOT(W), PER = 32 / SLOT;
  constexpr uint64_t SMASK = SLOT == 32 ? 0xffffffffull : 0xffffull;
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < COMB_WORDS(W, NDIG); i++) out[i] = 0;
#pragma unroll
  for (int i = 0; i < NDIG; i++) {
    const int bit = W * i, wd = bit >> 5, sh = bit & 31;
    uint64_t x = wd < 8 ? s[wd] : 0u;
    if (wd + 1 < 8) x |= (uint64_t)s[wd + 1] << 32;
    const uint32_t e = (uint32_t)((x >> sh) & ((1ull << W) - 1)) + carry;
    carry = e >= (1u << (W - 1)) ? 1u : 0u;
    const uint32_t d = (uint32_t)(((uint64_t)e - ((uint64_t)carry << W)) & SMASK);   /* two's complement slot */
    out[i / PER] |= d << (SLOT * (i % PER));
  }
}

}  // namespace fdgpu
