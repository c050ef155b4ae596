// Issue rate of v_cndmask_b32 on gfx950, settling the round-1 anomaly
// (profiles/r01_ubench_int.jsonl: 11 lane-ops/CU/clk for v_cndmask_b32 vs
// 111 for v_add_u32, where that ubench read VCC without declaring it).
// 8 independent chains per lane, 2 and 8 waves per SIMD:
//   e64  v_cndmask_b32 with the lane mask in an SGPR pair (declared operand)
//   vcc  v_cndmask_b32 with the mask in VCC (set by an s_mov_b64 in the same block)
//   add  v_add_u32 (reference full-rate instruction)
//   bfi  v_bfi_b32 with a per-lane all-ones/zero mask (a select without a lane mask)
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_sel.hip -o tools/ubench_sel
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 4096, CHAINS = 8;

template <int OP>
__global__ void __launch_bounds__(256) kbench(uint32_t *out, int seed) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x[CHAINS];
#pragma unroll
  for (int k = 0; k < CHAINS; k++) x[k] = tid * (k + 3) + seed;
  const uint32_t a = tid ^ 0x5a5a5a5au;
  const uint64_t m = __ballot((tid & 3u) == 1u);
  const uint32_t lm = (tid & 1u) ? 0xffffffffu : 0u;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int k = 0; k < CHAINS; k++) {
      if constexpr (OP == 0) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x[k]) : "v"(a), "s"(m));
      else if constexpr (OP == 1) asm volatile("s_mov_b64 vcc, %2\n v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x[k]) : "v"(a), "s"(m) : "vcc");
      else if constexpr (OP == 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[k]) : "v"(a));
      else asm volatile("v_bfi_b32 %0, %1, %2, %0" : "+v"(x[k]) : "v"(lm), "v"(a));
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < CHAINS; k++) s += x[k];
  out[tid] = s;
}

static const char *names[] = {"v_cndmask_b32_e64(sgpr mask)", "v_cndmask_b32_e32(vcc)", "v_add_u32", "v_bfi_b32"};

template <int OP>
static void run(uint32_t *d, int ncu, int waves) {
  const int blocks = ncu * waves, threads = 256;
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  kbench<OP><<<blocks, threads>>>(d, 1); CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    CHECK(hipEventRecord(e0)); kbench<OP><<<blocks, threads>>>(d, 2 + r); CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1)); float ms; CHECK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
  }
  const double lane_ops = (double)blocks * threads * ITERS * CHAINS;
  printf("{\"instr\": \"%s\", \"waves_per_simd\": %d, \"lane_ops_per_cu_per_clk_at_2.4GHz\": %.2f, \"ms\": %.4f}\n",
         names[OP], waves, lane_ops / (best * 1e-3) / (ncu * 2.4e9), best);
}

int main() {
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  uint32_t *d; CHECK(hipMalloc(&d, (size_t)p.multiProcessorCount * 8 * 256 * 4));
  for (int w : {2, 8}) { run<0>(d, p.multiProcessorCount, w); run<1>(d, p.multiProcessorCount, w);
                         run<2>(d, p.multiProcessorCount, w); run<3>(d, p.multiProcessorCount, w); }
  return 0;
}
