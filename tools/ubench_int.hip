// Integer VALU throughput microbenchmark for gfx950 (MI355X).
//
// Measures the chip-wide issue rate of the instructions a GF(2^255-19)
// field multiply can be built from, so that the limb representation and
// the VALU roofline (`r_mad`) rest on measured numbers:
//
//   mad_u64_u32   v_mad_u64_u32     32x32+64 -> 64 (radix-2^32 limbs)
//   mul_lo_u32    v_mul_lo_u32      32x32 -> low 32
//   mul_hi_u32    v_mul_hi_u32      32x32 -> high 32
//   mad_u32_u24   v_mad_u32_u24     24x24+32 -> low 32
//   mul_hi_u24    v_mul_hi_u32_u24  24x24 -> high 16
//   add_co        v_add_co_u32 + v_addc_co_u32 (one 64-bit add = 2 instr)
//   add_u32       v_add_u32
//   fma_f64       v_fma_f64
//
// Every instruction is issued through inline asm on 8 independent
// accumulator chains per lane, so the count is exact and the loop is
// throughput-bound.  Output: one JSON line per instruction with the
// lane-operations per second across the whole chip and per CU per clock.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_int.hip -o tools/ubench_int
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 32768;
constexpr int CHAINS = 8;

template <int OP>
__global__ void __launch_bounds__(256) kbench(uint32_t* out, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x, b = seed * 7u + blockIdx.x;
  uint64_t acc[CHAINS];
  double   dacc[CHAINS];
  uint32_t acc32[CHAINS];
#pragma unroll
  for (int k = 0; k < CHAINS; k++) { acc[k] = a + k; dacc[k] = (double)(a + k); acc32[k] = b + k; }
  double da = (double)a * 1e-9, db = (double)b * 1e-9;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int k = 0; k < CHAINS; k++) {
      if constexpr (OP == 0) {
        uint64_t cy;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cy) : "v"(a), "v"(b));
      } else if constexpr (OP == 1) {
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc32[k]) : "v"(a));
      } else if constexpr (OP == 2) {
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc32[k]) : "v"(a));
      } else if constexpr (OP == 3) {
        asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc32[k]) : "v"(a), "v"(b));
      } else if constexpr (OP == 4) {
        asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(acc32[k]) : "v"(a));
      } else if constexpr (OP == 5) {
        // one 64-bit add = v_add_co_u32 + v_addc_co_u32 (counted as 2 ops)
        uint32_t lo = (uint32_t)acc[k], hi = (uint32_t)(acc[k] >> 32);
        asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %3, vcc"
                     : "+v"(lo), "+v"(hi) : "v"(a), "v"(b) : "vcc");
        acc[k] = ((uint64_t)hi << 32) | lo;
      } else if constexpr (OP == 6) {
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc32[k]) : "v"(a));
      } else if constexpr (OP == 7) {
        asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(dacc[k]) : "v"(da), "v"(db));
      } else if constexpr (OP == 8) {
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[k]) : "v"((uint64_t)a));
      } else if constexpr (OP == 9) {
        asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(acc[k]));
      } else if constexpr (OP == 10) {
        uint32_t lo = (uint32_t)acc[k]; uint64_t cy;
        asm volatile("v_add_co_u32 %0, %1, %0, %2" : "+v"(lo), "=s"(cy) : "v"(a));
        acc[k] = (acc[k] & ~0xffffffffull) | lo;
      } else if constexpr (OP == 11) {
        asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(acc32[k]) : "v"(a));
      } else if constexpr (OP == 12) {
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(acc32[k]) : "v"(a));
      } else if constexpr (OP == 13) {
        asm volatile("v_mov_b32 %0, %1" : "=v"(acc32[k]) : "v"(a + k));
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CHAINS; k++) s += acc[k] + acc32[k] + (uint64_t)dacc[k];
  if (s == 0x123456789ull) out[0] = (uint32_t)s;  // keep live
}

static const char* names[] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u32_u24",
                              "v_mul_hi_u32_u24", "v_add_co_u32+v_addc_co_u32(vcc chain)", "v_add_u32", "v_fma_f64",
                              "v_lshl_add_u64", "v_lshrrev_b64", "v_add_co_u32(sgpr carry)", "v_alignbit_b32",
                              "v_cndmask_b32", "v_mov_b32"};
static const int ops_per_chain[] = {1, 1, 1, 1, 1, 2, 1, 1, 1, 1, 1, 1, 1, 1};

template <int OP>
static void run(uint32_t* d, int ncu, double clk_ghz) {
  const int blocks = ncu * 8, threads = 256;  // 8 waves/SIMD worth of 256-thread blocks
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  kbench<OP><<<blocks, threads>>>(d, 1);  // warm
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    CHECK(hipEventRecord(e0));
    kbench<OP><<<blocks, threads>>>(d, 2 + r);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  double lane_ops = (double)blocks * threads * ITERS * CHAINS * ops_per_chain[OP];
  double rate = lane_ops / (best * 1e-3);
  printf("{\"instr\": \"%s\", \"lane_ops_per_s\": %.4e, \"lane_ops_per_cu_per_clk_at_%.1fGHz\": %.2f, \"ms\": %.3f}\n",
         names[OP], rate, clk_ghz, rate / (ncu * clk_ghz * 1e9), best);
  CHECK(hipEventDestroy(e0)); CHECK(hipEventDestroy(e1));
}

int main() {
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  int ncu = p.multiProcessorCount;
  double clk = p.clockRate / 1e6;
  printf("{\"device\": \"%s\", \"gcn_arch\": \"%s\", \"cus\": %d, \"clock_ghz\": %.3f}\n", p.name, p.gcnArchName, ncu, clk);
  uint32_t* d; CHECK(hipMalloc(&d, 64));
  run<0>(d, ncu, clk); run<1>(d, ncu, clk); run<2>(d, ncu, clk); run<3>(d, ncu, clk);
  run<4>(d, ncu, clk); run<5>(d, ncu, clk); run<6>(d, ncu, clk); run<7>(d, ncu, clk);
  run<8>(d, ncu, clk); run<9>(d, ncu, clk); run<10>(d, ncu, clk); run<11>(d, ncu, clk);
  run<12>(d, ncu, clk); run<13>(d, ncu, clk);
  CHECK(hipFree(d));
  return 0;
}
