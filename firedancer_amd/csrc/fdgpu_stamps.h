/* fdgpu_stamps.h -- per-phase cycle stamps of the verify kernel (a
   diagnostic build only: -DFDGPU_PHASE_STAMPS=1, see tools/phase_stamps.py).
   In the product build FDGPU_STAMP(i) compiles to nothing.

   Lane 0 of each wave records the shader clock (s_memtime) at phase
   boundary i into g_fdgpu_stamps[wave][i] with an ordinary vector store;
   fdgpu_debug_stamps copies the table out.  Nothing the kernel computes
   reads the stamps. */
#pragma once

#define FDGPU_STAMP_SLOTS 10u      /* 0..7 shader clock at the phase boundaries; 8, 9 the
                                      constant 100-MHz clock at boundaries 0 and 7 */
#define FDGPU_STAMP_WAVES (1u << 15)     /* covers 2M signatures */

#if FDGPU_PHASE_STAMPS
__device__ uint64_t g_fdgpu_stamps[FDGPU_STAMP_WAVES * FDGPU_STAMP_SLOTS];

__device__ __forceinline__ void fdgpu_stamp(uint32_t slot) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t t = __builtin_amdgcn_s_memtime();
  const uint64_t rt = (slot == 0 || slot == 7) ? __builtin_amdgcn_s_memrealtime() : 0;
  volatile uint64_t *row = g_fdgpu_stamps + (size_t)(wave % FDGPU_STAMP_WAVES) * FDGPU_STAMP_SLOTS;
  if (lane == 0) {
    row[slot] = t;
    if (slot == 0) row[8] = rt;
    if (slot == 7) row[9] = rt;
  }
}
#define FDGPU_STAMP(i) fdgpu_stamp(i)
#else
#define FDGPU_STAMP(i) do {} while (0)
#endif
