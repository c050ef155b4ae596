// PCIe bandwidth of kernel loads and stores to pinned host memory on MI355X
// (the gathered tile batches read payloads and write out frags this way),
// next to the DMA engines' copies (hipMemcpyAsync).  Each row: GB/s for
// `mb` MB moved by `blocks` x 256 threads, 16-B accesses, `unroll` loads in
// flight per lane (reads), or one store per lane per step (writes).
//
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_pcie.hip -o tools/ubench_pcie && tools/ubench_pcie
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <int U>
__global__ void __launch_bounds__(256) rd(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x * U;
  for (size_t i = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x; i < n; i += stride) {
    uint4 v[U];
#pragma unroll
    for (int j = 0; j < U; j++) v[j] = i + (size_t)j * blockDim.x < n ? src[i + (size_t)j * blockDim.x] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < U; j++) if (i + (size_t)j * blockDim.x < n) dst[i + (size_t)j * blockDim.x] = v[j];
  }
}

__global__ void __launch_bounds__(256) wr(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) dst[i] = src[i];
}

static float time_ms(hipEvent_t a, hipEvent_t b) { float ms; CHK(hipEventSynchronize(b)); CHK(hipEventElapsedTime(&ms, a, b)); return ms; }

int main() {
  const size_t mb = 64, bytes = mb << 20, n = bytes / 16;
  uint4 *h, *d;
  CHK(hipHostMalloc((void **)&h, bytes, hipHostMallocDefault));
  CHK(hipMalloc((void **)&d, bytes));
  memset(h, 1, bytes);
  uint4 *hd;
  CHK(hipHostGetDevicePointer((void **)&hd, h, 0));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  const int iters = 10;
  printf("{\"what\": \"dma_h2d\", \"mb\": %zu, ", mb);
  CHK(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
  CHK(hipEventRecord(a)); for (int i = 0; i < iters; i++) CHK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, 0)); CHK(hipEventRecord(b));
  printf("\"gbps\": %.2f}\n", bytes * iters / (time_ms(a, b) * 1e-3) / 1e9);
  printf("{\"what\": \"dma_d2h\", \"mb\": %zu, ", mb);
  CHK(hipEventRecord(a)); for (int i = 0; i < iters; i++) CHK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, 0)); CHK(hipEventRecord(b));
  printf("\"gbps\": %.2f}\n", bytes * iters / (time_ms(a, b) * 1e-3) / 1e9);
  for (int blocks : {16, 64, 256, 1024}) {
    for (int u : {1, 4}) {
      auto launch = [&]() {
        if (u == 1) hipLaunchKernelGGL(rd<1>, dim3(blocks), dim3(256), 0, 0, hd, d, n);
        else hipLaunchKernelGGL(rd<4>, dim3(blocks), dim3(256), 0, 0, hd, d, n);
      };
      launch();
      CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(a)); for (int i = 0; i < iters; i++) launch(); CHK(hipEventRecord(b));
      printf("{\"what\": \"kernel_read_host\", \"blocks\": %d, \"unroll\": %d, \"gbps\": %.2f}\n", blocks, u,
             bytes * iters / (time_ms(a, b) * 1e-3) / 1e9);
    }
    hipLaunchKernelGGL(wr, dim3(blocks), dim3(256), 0, 0, d, hd, n);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a)); for (int i = 0; i < iters; i++) hipLaunchKernelGGL(wr, dim3(blocks), dim3(256), 0, 0, d, hd, n); CHK(hipEventRecord(b));
    printf("{\"what\": \"kernel_write_host\", \"blocks\": %d, \"gbps\": %.2f}\n", blocks, bytes * iters / (time_ms(a, b) * 1e-3) / 1e9);
  }
  // both directions at once: a read kernel and a write kernel on two streams
  hipStream_t s1, s2;
  CHK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking)); CHK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  uint4 *d2; CHK(hipMalloc((void **)&d2, bytes));
  uint4 *h2, *hd2; CHK(hipHostMalloc((void **)&h2, bytes, hipHostMallocDefault)); CHK(hipHostGetDevicePointer((void **)&hd2, h2, 0));
  CHK(hipDeviceSynchronize());
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; i++) {
    hipLaunchKernelGGL(rd<4>, dim3(64), dim3(256), 0, s1, hd, d, n);
    hipLaunchKernelGGL(wr, dim3(64), dim3(256), 0, s2, d2, hd2, n);
  }
  CHK(hipDeviceSynchronize());
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("{\"what\": \"kernel_read_and_write_host\", \"blocks\": 64, \"gbps_each\": %.2f}\n", bytes * iters / sec / 1e9);
  return 0;
}
