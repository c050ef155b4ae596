/* fdt_hash.h -- fd_hash (src/util/fd_hash.c:12-73, xxhash-r39 over 64-bit
   lanes) as one source for the host and the GPU: g++ builds it into
   libfd_verify_tile.so (fdt_hash, the tile's dedup tag), hipcc into the
   frag-batch finish kernel, which tags each parsed transaction's first
   signature on the device (fdgpu_submit_frags_io). */
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define FDT_HASH_HD __host__ __device__ __forceinline__
#else
#define FDT_HASH_HD static inline
#endif

#define FDT_HASH_P1 11400714785074694791ULL
#define FDT_HASH_P2 14029467366897019727ULL
#define FDT_HASH_P3 1609587929392839161ULL
#define FDT_HASH_P4 9650029242287828579ULL
#define FDT_HASH_P5 2870177450012600261ULL

FDT_HASH_HD uint64_t fdt_hash_rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
/* unaligned little-endian loads, byte by byte (the device reads payload
   bytes at any offset) */
FDT_HASH_HD uint64_t fdt_hash_rd(const uint8_t *p, int n) {
  uint64_t v = 0;
  for (int i = 0; i < n; i++) v |= (uint64_t)p[i] << (8 * i);
  return v;
}
FDT_HASH_HD uint64_t fdt_hash_round(uint64_t acc, uint64_t in) {
  return fdt_hash_rotl(acc + in * FDT_HASH_P2, 31) * FDT_HASH_P1;
}
FDT_HASH_HD uint64_t fdt_hash_merge(uint64_t h, uint64_t acc) {
  return (h ^ fdt_hash_round(0, acc)) * FDT_HASH_P1 + FDT_HASH_P4;
}

FDT_HASH_HD uint64_t fdt_hash_core(uint64_t seed, const uint8_t *p, uint64_t sz) {
  const uint8_t *end = p + sz;
  uint64_t h;
  if (sz >= 32) {
    uint64_t a = seed + FDT_HASH_P1 + FDT_HASH_P2, b = seed + FDT_HASH_P2, c = seed, d = seed - FDT_HASH_P1;
    do {
      a = fdt_hash_round(a, fdt_hash_rd(p, 8));
      b = fdt_hash_round(b, fdt_hash_rd(p + 8, 8));
      c = fdt_hash_round(c, fdt_hash_rd(p + 16, 8));
      d = fdt_hash_round(d, fdt_hash_rd(p + 24, 8));
      p += 32;
    } while (p + 32 <= end);
    h = fdt_hash_rotl(a, 1) + fdt_hash_rotl(b, 7) + fdt_hash_rotl(c, 12) + fdt_hash_rotl(d, 18);
    h = fdt_hash_merge(h, a);
    h = fdt_hash_merge(h, b);
    h = fdt_hash_merge(h, c);
    h = fdt_hash_merge(h, d);
  } else {
    h = seed + FDT_HASH_P5;
  }
  h += sz;
  for (; p + 8 <= end; p += 8) h = fdt_hash_rotl(h ^ fdt_hash_round(0, fdt_hash_rd(p, 8)), 27) * FDT_HASH_P1 + FDT_HASH_P4;
  if (p + 4 <= end) {
    h = fdt_hash_rotl(h ^ (fdt_hash_rd(p, 4) * FDT_HASH_P1), 23) * FDT_HASH_P2 + FDT_HASH_P3;
    p += 4;
  }
  for (; p < end; p++) h = fdt_hash_rotl(h ^ ((uint64_t)*p * FDT_HASH_P5), 11) * FDT_HASH_P1;
  h ^= h >> 33;
  h *= FDT_HASH_P2;
  h ^= h >> 29;
  h *= FDT_HASH_P3;
  h ^= h >> 32;
  return h;
}
