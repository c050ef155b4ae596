// Carry-scheme microbenchmark for the radix-2^25.5 field product on gfx950.
//
//   cur  fdgpu_fe.h as shipped: 10 independent 64-bit column sums, then a
//        12-step two-chain carry (shift + mask + 64-bit add per step)
//   ff   "feed-forward": columns summed in order 0..9, each column's mad chain
//        starts from the previous column's carry, so the carry add rides in
//        the v_mad_u64_u32 addend (one long dependent chain per product)
//
//   ffa  feed-forward with each v_mad_u64_u32 in inline asm, so the compiler
//        cannot re-associate the column chain and add the carry separately
//
// One product chain per lane (x <- x*y or x <- x^2), 2 waves per SIMD, with
// the engine's scheduling fence after each product, as in the verify kernel.
// Results are canonicalised on the device and compared between schemes.
// Build (cur = the two-chain scheme): hipcc --offload-arch=gfx950 -O3 -DFDGPU_FE_FF=0 tools/ubench_carry.hip -o tools/ubench_carry
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../firedancer_amd/csrc/fdgpu_fe.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

using namespace fdgpu;

FDG_DEV void fe_mul_ff(fe &h, const fe &f, const fe &g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) { g19[i] = 19u * g.v[i]; f2[i] = f.v[i] << 1; }
  uint64_t carry = 0;
  uint32_t r[10];                  /* h may alias f: write it only at the end */
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t s = carry;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      int j = k - i;
      const bool wrap = j < 0;
      if (wrap) j += 10;
      const bool dbl = (i & 1) && (j & 1);
      s += (uint64_t)(dbl ? f2[i] : f.v[i]) * (wrap ? g19[j] : g.v[j]);
    }
    const int bits = (k & 1) ? 25 : 26;
    r[k] = (uint32_t)s & ((1u << bits) - 1);
    carry = s >> bits;
  }
  const uint64_t t = (uint64_t)r[0] + carry * 19u;
  r[0] = (uint32_t)t & ((1u << 26) - 1);
  r[1] += (uint32_t)(t >> 26);
#pragma unroll
  for (int k = 0; k < 10; k++) h.v[k] = r[k];
  FDG_SCHED_FENCE();
}

FDG_DEV void fe_sq_ff(fe &h, const fe &f) {
  uint32_t f2[10], f4[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) { f2[i] = f.v[i] << 1; f4[i] = f.v[i] << 2; f19[i] = 19u * f.v[i]; }
  uint64_t carry = 0;
  uint32_t r[10];                  /* h may alias f: write it only at the end */
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t s = carry;
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
      for (int j = i; j < 10; j++) {
        if ((i + j) % 10 != k) continue;
        const bool wrap = (i + j) >= 10;
        const int mul2 = (i != j ? 1 : 0) + (((i & 1) && (j & 1)) ? 1 : 0);
        const uint32_t a = mul2 == 0 ? f.v[i] : (mul2 == 1 ? f2[i] : f4[i]);
        s += (uint64_t)a * (wrap ? f19[j] : f.v[j]);
      }
    }
    const int bits = (k & 1) ? 25 : 26;
    r[k] = (uint32_t)s & ((1u << bits) - 1);
    carry = s >> bits;
  }
  const uint64_t t = (uint64_t)r[0] + carry * 19u;
  r[0] = (uint32_t)t & ((1u << 26) - 1);
  r[1] += (uint32_t)(t >> 26);
#pragma unroll
  for (int k = 0; k < 10; k++) h.v[k] = r[k];
  FDG_SCHED_FENCE();
}

FDG_DEV uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=&v"(r), "=s"(cc) : "v"(a), "v"(b), "v"(c));
  (void)cc;
  return r;
}

FDG_DEV void fe_mul_ffa(fe &h, const fe &f, const fe &g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) { g19[i] = 19u * g.v[i]; f2[i] = f.v[i] << 1; }
  uint64_t carry = 0;
  uint32_t r[10];                  /* h may alias f: write it only at the end */
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t s = carry;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      int j = k - i;
      const bool wrap = j < 0;
      if (wrap) j += 10;
      const bool dbl = (i & 1) && (j & 1);
      s = mad64(dbl ? f2[i] : f.v[i], wrap ? g19[j] : g.v[j], s);
    }
    const int bits = (k & 1) ? 25 : 26;
    r[k] = (uint32_t)s & ((1u << bits) - 1);
    carry = s >> bits;
  }
  const uint64_t t = (uint64_t)r[0] + carry * 19u;
  r[0] = (uint32_t)t & ((1u << 26) - 1);
  r[1] += (uint32_t)(t >> 26);
#pragma unroll
  for (int k = 0; k < 10; k++) h.v[k] = r[k];
  FDG_SCHED_FENCE();
}

FDG_DEV void fe_sq_ffa(fe &h, const fe &f) {
  uint32_t f2[10], f4[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) { f2[i] = f.v[i] << 1; f4[i] = f.v[i] << 2; f19[i] = 19u * f.v[i]; }
  uint64_t carry = 0;
  uint32_t r[10];                  /* h may alias f: write it only at the end */
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t s = carry;
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
      for (int j = i; j < 10; j++) {
        if ((i + j) % 10 != k) continue;
        const bool wrap = (i + j) >= 10;
        const int mul2 = (i != j ? 1 : 0) + (((i & 1) && (j & 1)) ? 1 : 0);
        const uint32_t a = mul2 == 0 ? f.v[i] : (mul2 == 1 ? f2[i] : f4[i]);
        s = mad64(a, wrap ? f19[j] : f.v[j], s);
      }
    }
    const int bits = (k & 1) ? 25 : 26;
    r[k] = (uint32_t)s & ((1u << bits) - 1);
    carry = s >> bits;
  }
  const uint64_t t = (uint64_t)r[0] + carry * 19u;
  r[0] = (uint32_t)t & ((1u << 26) - 1);
  r[1] += (uint32_t)(t >> 26);
#pragma unroll
  for (int k = 0; k < 10; k++) h.v[k] = r[k];
  FDG_SCHED_FENCE();
}

// V: 0 cur mul, 1 ff mul, 2 cur sq, 3 ff sq, 4 ffa mul, 5 ffa sq
template <int V>
__global__ void __launch_bounds__(256) kbench(uint32_t *out, const uint32_t *in, int iters) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  fe x, y;
#pragma unroll
  for (int w = 0; w < 10; w++) { x.v[w] = in[w * 64 + (gid & 63)]; y.v[w] = in[(10 + w) * 64 + (gid & 63)]; }
  for (int it = 0; it < iters; it++) {
    if constexpr (V == 0) fe_mul(x, x, y);
    else if constexpr (V == 1) fe_mul_ff(x, x, y);
    else if constexpr (V == 2) fe_sq(x, x);
    else if constexpr (V == 3) fe_sq_ff(x, x);
    else if constexpr (V == 4) fe_mul_ffa(x, x, y);
    else fe_sq_ffa(x, x);
  }
  fe_canon(x);
#pragma unroll
  for (int w = 0; w < 10; w++) out[(size_t)gid * 10 + w] = x.v[w];
}

template <int V>
static double run(uint32_t *dout, const uint32_t *din, int ncu, int iters, uint32_t *canon) {
  const int blocks = ncu * 8, threads = 256;
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  kbench<V><<<blocks, threads>>>(dout, din, 2); CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    CHECK(hipEventRecord(e0)); kbench<V><<<blocks, threads>>>(dout, din, iters); CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1)); float ms; CHECK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
  }
  kbench<V><<<1, 64>>>(dout, din, 37); CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(canon, dout, 64 * 10 * 4, hipMemcpyDeviceToHost));
  return (double)blocks * threads * iters / (best * 1e-3);
}

int main() {
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  uint32_t hin[20 * 64];
  srand(7);
  for (int i = 0; i < 20 * 64; i++) hin[i] = ((uint32_t)rand() ^ ((uint32_t)rand() << 16)) & (((i / 64) & 1) ? 0x1ffffff : 0x3ffffff);
  uint32_t *din, *dout;
  CHECK(hipMalloc(&din, sizeof(hin)));
  CHECK(hipMemcpy(din, hin, sizeof(hin), hipMemcpyHostToDevice));
  CHECK(hipMalloc(&dout, (size_t)ncu * 8 * 256 * 10 * 4));
  const int iters = 2048;
  static uint32_t c0[640], c1[640], c2[640], c3[640], c4[640], c5[640];
  const double r0 = run<0>(dout, din, ncu, iters, c0), r1 = run<1>(dout, din, ncu, iters, c1);
  const double r2 = run<2>(dout, din, ncu, iters, c2), r3 = run<3>(dout, din, ncu, iters, c3);
  const double r4 = run<4>(dout, din, ncu, iters, c4), r5 = run<5>(dout, din, ncu, iters, c5);
  printf("{\"eq01\": %d, \"eq04\": %d, \"eq23\": %d, \"eq25\": %d, \"c0\": [%u, %u, %u], \"c1\": [%u, %u, %u], \"c4\": [%u, %u, %u]}\n",
         !memcmp(c0, c1, sizeof(c0)), !memcmp(c0, c4, sizeof(c0)), !memcmp(c2, c3, sizeof(c2)), !memcmp(c2, c5, sizeof(c2)),
         c0[0], c0[1], c0[9], c1[0], c1[1], c1[9], c4[0], c4[1], c4[9]);
  const int agree_mul = !memcmp(c0, c1, sizeof(c0)) && !memcmp(c0, c4, sizeof(c0));
  const int agree_sq = !memcmp(c2, c3, sizeof(c2)) && !memcmp(c2, c5, sizeof(c2));
  printf("{\"mul_ffa_per_s\": %.4e, \"mul_ffa_gain\": %.4f, \"sq_ffa_per_s\": %.4e, \"sq_ffa_gain\": %.4f}\n", r4, r4 / r0 - 1, r5, r5 / r2 - 1);
  printf("{\"mul_cur_per_s\": %.4e, \"mul_ff_per_s\": %.4e, \"mul_gain\": %.4f, \"agree_mul\": %d}\n", r0, r1, r1 / r0 - 1, agree_mul);
  printf("{\"sq_cur_per_s\": %.4e, \"sq_ff_per_s\": %.4e, \"sq_gain\": %.4f, \"agree_sq\": %d}\n", r2, r3, r3 / r2 - 1, agree_sq);
  return agree_mul && agree_sq ? 0 : 1;
}
