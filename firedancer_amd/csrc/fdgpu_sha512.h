/* fdgpu_sha512.h -- one-message-per-lane SHA-512 (FIPS 180-4) on gfx950.

   Computes k' = SHA-512(R || A || M) for the verify path (the reference's
   fd_sha512_init/append/fini sequence at fd_ed25519_user.c:205-206 /
   :283-285; core fd_sha512.c:264-399).  The 64-bit state lives in VGPR
   pairs; rotations lower to v_alignbit_b32 pairs, additions to
   v_add_co/v_addc.  Blocks are assembled per lane from R/A (registers) and
   the message bytes in the batch arena (aligned dword loads + byte
   funnel shifts), padded and length-terminated in registers: there is no
   staging copy of the message.  Lanes whose message needs fewer blocks
   than the wave's longest simply idle through the extra blocks (the host
   groups signatures by block count). */
#pragma once

#include "fdgpu_fe.h"

namespace fdgpu {

__constant__ static const uint64_t SHA512_K[80] = {
  0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
  0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
  0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
  0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
  0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
  0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
  0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
  0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
  0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
  0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
  0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
  0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
  0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
  0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
  0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
  0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
  0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
  0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
  0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
  0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL,
};

/* 64-bit rotate / shift as two v_alignbit_b32 (funnel shifts of the two
   halves; r is a compile-time constant in every use); the generic lowering
   is four 64-bit shifts and ors */
FDG_DEV uint64_t rotr64(uint64_t x, int r) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  const uint32_t a = r < 32 ? hi : lo, b = r < 32 ? lo : hi, n = (uint32_t)(r & 31);
  return ((uint64_t)__builtin_amdgcn_alignbit(b, a, n) << 32) | __builtin_amdgcn_alignbit(a, b, n);
}
/* majority of three bits, one v_bitop3_b32 per half (truth table 0xE8,
   symmetric in its inputs) */
FDG_DEV uint64_t maj64(uint64_t a, uint64_t b, uint64_t c) {
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0xE8);
  const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0xE8);
  return ((uint64_t)hi << 32) | lo;
}
FDG_DEV uint64_t shr64(uint64_t x, int r) {           /* r < 32 */
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return ((uint64_t)(hi >> r) << 32) | __builtin_amdgcn_alignbit(hi, lo, (uint32_t)r);
}
/* a ^ b ^ c as one gfx950 v_bitop3_b32 per half (truth table 0x96: the
   parity of the three inputs); the compiler emits two v_xor_b32 otherwise */
FDG_DEV uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0x96);
  const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0x96);
  return ((uint64_t)hi << 32) | lo;
}
FDG_DEV uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

FDG_DEV void sha512_compress(uint64_t (&h)[8], uint64_t (&w)[16]) {
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int r = 0; r < 80; r += 16) {
#pragma unroll
    for (int t = 0; t < 16; t++) {
      if (r) {
        const uint64_t w15 = w[(t + 1) & 15], w2 = w[(t + 14) & 15];
        const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), shr64(w15, 7));
        const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), shr64(w2, 6));
        w[t] += s0 + w[(t + 9) & 15] + s1;
      }
      const uint64_t S1 = xor3_64(rotr64(e, 14), rotr64(e, 18), rotr64(e, 41));
      const uint64_t ch = (e & f) ^ (~e & g);
      const uint64_t t1 = hh + S1 + ch + SHA512_K[r + t] + w[t];
      const uint64_t S0 = xor3_64(rotr64(a, 28), rotr64(a, 34), rotr64(a, 39));
      const uint64_t maj = maj64(a, b, c);
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + maj;
    }
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

/* Little-endian u32 at byte address p (any alignment), from two aligned
   dword loads and a funnel shift.  Pointer arithmetic (not integer casts)
   keeps the global address space visible to the compiler (global_load, not
   flat_load). */
FDG_DEV uint32_t load_u32_unaligned(const uint8_t *p) {
  const uint32_t mis = (uint32_t)((uintptr_t)p & 3u);
  const uint32_t *q = (const uint32_t *)(p - mis);
  const uint32_t lo = q[0], hi = q[1];
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8u * mis));
}

/* Message part of one SHA block: words w[t0..15] take message bytes
   [base + 8 (t - t0), +8) as big-endian words (base >= 0).  The lane loads
   the aligned dwords covering the range once and funnel-shifts them; bytes at
   or beyond msg_sz become the 0x80 pad and zeros.  Loads are unconditional:
   when the whole range lies past the message, the load base is clamped to the
   message start (the words are then fully masked), and the arena carries
   FDGPU_ARENA_SLACK (>= 132) readable bytes past its end. */
template <int T0>
FDG_DEV void msg_block(uint64_t (&w)[16], const uint8_t *msg, uint32_t msg_sz, uint32_t base) {
  constexpr int NW = 16 - T0;                 /* message words in this block */
  const uint32_t lb = base < msg_sz ? base : 0u;
  const uint8_t *p = msg + lb;
  const uint32_t mis = (uint32_t)((uintptr_t)p & 3u);
  const uint32_t *q = (const uint32_t *)(p - mis);
  uint32_t d[2 * NW + 1];
#pragma unroll
  for (int i = 0; i < 2 * NW + 1; i++) d[i] = q[i];
#pragma unroll
  for (int u = 0; u < NW; u++) {
    const uint32_t lo = (uint32_t)((((uint64_t)d[2 * u + 1] << 32) | d[2 * u]) >> (8u * mis));
    const uint32_t hi = (uint32_t)((((uint64_t)d[2 * u + 2] << 32) | d[2 * u + 1]) >> (8u * mis));
    uint64_t v = ((uint64_t)hi << 32) | lo;
    const int64_t rem = (int64_t)msg_sz - (int64_t)base - 8 * u;   /* valid bytes in this word */
    if (rem < 8) {
      const int n = rem < 0 ? 0 : (int)rem;
      v = n ? (v & ((~0ull) >> (64 - 8 * n))) : 0ull;
      if (rem >= 0) v |= 0x80ull << (8 * n);
    }
    w[T0 + u] = ((uint64_t)bswap32((uint32_t)v) << 32) | bswap32((uint32_t)(v >> 32));
  }
}

FDG_DEV uint32_t sha512_hram_blocks(uint32_t msg_sz) { return (64u + msg_sz + 16u) / 128u + 1u; }

/* digest (as 8 big-endian-state words) of R(32) || A(32) || msg(msg_sz).
   nblk_wave: max block count over the wave (uniform loop bound). */
FDG_DEV void sha512_hram(uint64_t (&h)[8], const uint32_t (&R)[8], const uint32_t (&A)[8],
                         const uint8_t *msg, uint32_t msg_sz, uint32_t nblk_wave) {
  const uint64_t H0[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                          0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                          0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
#pragma unroll
  for (int i = 0; i < 8; i++) h[i] = H0[i];
  const uint32_t nblk = sha512_hram_blocks(msg_sz);
  const uint64_t bitlen = (uint64_t)(64u + msg_sz) * 8u;
  for (uint32_t blk = 0; blk < nblk_wave; blk++) {
    uint64_t w[16];
    if (blk == 0) {
      msg_block<8>(w, msg, msg_sz, 0u);
#pragma unroll
      for (int t = 0; t < 4; t++) w[t] = ((uint64_t)bswap32(R[2 * t]) << 32) | bswap32(R[2 * t + 1]);
#pragma unroll
      for (int t = 0; t < 4; t++) w[4 + t] = ((uint64_t)bswap32(A[2 * t]) << 32) | bswap32(A[2 * t + 1]);
    } else {
      msg_block<0>(w, msg, msg_sz, 128u * blk - 64u);
    }
    if (blk + 1 == nblk) { w[14] = 0; w[15] = bitlen; }
    uint64_t hs[8];
#pragma unroll
    for (int i = 0; i < 8; i++) hs[i] = h[i];
    sha512_compress(hs, w);
    if (blk < nblk) {
#pragma unroll
      for (int i = 0; i < 8; i++) h[i] = hs[i];
    }
  }
}

/* Plain SHA-512 of msg (used by the hash-only test/bench kernel). */
FDG_DEV void sha512_plain(uint64_t (&h)[8], const uint8_t *msg, uint32_t msg_sz, uint32_t nblk_wave) {
  const uint64_t H0[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                          0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                          0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
#pragma unroll
  for (int i = 0; i < 8; i++) h[i] = H0[i];
  const uint32_t nblk = (msg_sz + 16u) / 128u + 1u;
  const uint64_t bitlen = (uint64_t)msg_sz * 8u;
  for (uint32_t blk = 0; blk < nblk_wave; blk++) {
    uint64_t w[16];
    msg_block<0>(w, msg, msg_sz, 128u * blk);
    if (blk + 1 == nblk) { w[14] = 0; w[15] = bitlen; }
    uint64_t hs[8];
#pragma unroll
    for (int i = 0; i < 8; i++) hs[i] = h[i];
    sha512_compress(hs, w);
    if (blk < nblk) {
#pragma unroll
      for (int i = 0; i < 8; i++) h[i] = hs[i];
    }
  }
}

}  // namespace fdgpu
