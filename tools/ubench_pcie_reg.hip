// H2D rate of a host arena the engine DMAs in place (fdgpu_host_register ->
// hipHostRegister of the caller's malloc'd pages) against a pinned
// hipHostMalloc buffer of the same size: one copy on one stream, the same
// bytes split over k streams, and a kernel reading the host memory.  The
// registered host-fed line (bench.py host_fed_registered_*) moves 364 MB a
// batch this way.
//
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_pcie_reg.hip -o tools/ubench_pcie_reg && tools/ubench_pcie_reg
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <chrono>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void __launch_bounds__(256) rd4(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x * 4;
  for (size_t i = (size_t)blockIdx.x * blockDim.x * 4 + threadIdx.x; i < n; i += stride) {
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) v[j] = i + (size_t)j * blockDim.x < n ? src[i + (size_t)j * blockDim.x] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; j++) if (i + (size_t)j * blockDim.x < n) dst[i + (size_t)j * blockDim.x] = v[j];
  }
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static void run(const char *what, uint8_t *h, uint8_t *d, size_t bytes, hipStream_t *st) {
  const int iters = 4;
  for (int k : {1, 2, 4, 8}) {
    CHK(hipDeviceSynchronize());
    const double t0 = now();
    for (int it = 0; it < iters; it++) {
      const size_t piece = (bytes / k + 4095) & ~(size_t)4095;
      for (int j = 0; j < k; j++) {
        const size_t off = (size_t)j * piece;
        if (off >= bytes) break;
        const size_t m = bytes - off < piece ? bytes - off : piece;
        CHK(hipMemcpyAsync(d + off, h + off, m, hipMemcpyHostToDevice, st[j]));
      }
    }
    CHK(hipDeviceSynchronize());
    printf("{\"what\": \"%s_dma_h2d\", \"mb\": %zu, \"streams\": %d, \"gbps\": %.2f}\n", what, bytes >> 20, k,
           bytes * (double)iters / (now() - t0) / 1e9);
  }
  uint8_t *hd;
  CHK(hipHostGetDevicePointer((void **)&hd, h, 0));
  for (int blocks : {64, 256}) {
    hipLaunchKernelGGL(rd4, dim3(blocks), dim3(256), 0, 0, (const uint4 *)hd, (uint4 *)d, bytes / 16);
    CHK(hipDeviceSynchronize());
    const double t0 = now();
    for (int it = 0; it < iters; it++)
      hipLaunchKernelGGL(rd4, dim3(blocks), dim3(256), 0, 0, (const uint4 *)hd, (uint4 *)d, bytes / 16);
    CHK(hipDeviceSynchronize());
    printf("{\"what\": \"%s_kernel_read\", \"mb\": %zu, \"blocks\": %d, \"gbps\": %.2f}\n", what, bytes >> 20, blocks,
           bytes * (double)iters / (now() - t0) / 1e9);
  }
}

int main() {
  const size_t bytes = 364ull << 20;
  uint8_t *d;
  CHK(hipMalloc((void **)&d, bytes));
  hipStream_t st[8];
  for (auto &s : st) CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  {
    uint8_t *h;
    CHK(hipHostMalloc((void **)&h, bytes, hipHostMallocDefault));
    memset(h, 1, bytes);
    run("pinned", h, d, bytes, st);
    CHK(hipHostFree(h));
  }
  for (int thp : {0, 1}) {
    uint8_t *h = (uint8_t *)aligned_alloc(2u << 20, bytes);
    if (thp) madvise(h, bytes, MADV_HUGEPAGE);
    memset(h, 1, bytes);
    CHK(hipHostRegister(h, bytes, hipHostRegisterMapped));
    run(thp ? "registered_thp" : "registered", h, d, bytes, st);
    CHK(hipHostUnregister(h));
    free(h);
  }
  return 0;
}
