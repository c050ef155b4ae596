// Which CUs (XCC id, CU id) a CU-masked stream's workgroups land on, for
// single-bit and strided masks; and the default stream's mask.
//   hipcc -O2 --offload-arch=gfx950 tools/probe_cumask.hip -o build/probe_cumask && build/probe_cumask
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>
#include <chrono>
#include <set>
#include <vector>

__global__ void where(uint32_t *out) {
  if (threadIdx.x == 0) {
    const uint32_t xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));   /* HW_REG_XCC_ID [3:0] */
    const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));     /* HW_REG_HW_ID (gfx9) */
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
}

int main() {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
  printf("cus %d\n", p.multiProcessorCount);
  hipStream_t s0;
  (void)hipStreamCreate(&s0);
  uint32_t m[16] = {0};
  if (hipExtStreamGetCUMask(s0, 16, m) == hipSuccess) {
    printf("default mask:");
    for (int i = 0; i < 16; i++) printf(" %08x", m[i]);
    printf("\n");
  }
  uint32_t *d, *h;
  (void)hipMalloc(&d, 4096 * 8);
  h = (uint32_t *)malloc(4096 * 8);
  std::vector<std::vector<int>> tests = {{0}, {1}, {7}, {8}, {31}, {32}, {0, 1, 2, 3, 4, 5, 6, 7}, {0, 32, 64, 96, 128, 160, 192, 224}};
  for (auto &bits : tests) {
    uint32_t mk[8] = {0};
    for (int b : bits) mk[b / 32] |= 1u << (b % 32);
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, 8, mk) != hipSuccess) { printf("create failed\n"); continue; }
    (void)hipMemsetAsync(d, 0xff, 4096 * 8, s);
    hipLaunchKernelGGL(where, dim3(512), dim3(64), 0, s, d);
    const auto t0 = std::chrono::steady_clock::now();
    while (hipStreamQuery(s) == hipErrorNotReady) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(3)) { printf("bits %d..: STUCK\n", bits[0]); fflush(stdout); _exit(3); }
      usleep(1000);
    }
    (void)hipMemcpy(h, d, 512 * 8, hipMemcpyDeviceToHost);
    std::set<std::pair<uint32_t, uint32_t>> cus;
    for (int i = 0; i < 512; i++) cus.insert({h[2 * i], (h[2 * i + 1] >> 8) & 0xf | ((h[2 * i + 1] >> 13) & 0x7) << 4 | ((h[2 * i + 1] >> 12) & 1) << 8});
    printf("bits");
    for (int b : bits) printf(" %d", b);
    printf(" -> %zu (xcc,cu/sh/se):", cus.size());
    for (auto &c : cus) printf(" (%u,%03x)", c.first, c.second);
    printf("\n");
    fflush(stdout);
    (void)hipStreamDestroy(s);
  }
  return 0;
}
