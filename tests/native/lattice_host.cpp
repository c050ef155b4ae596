// Host build of firedancer_amd/csrc/fdgpu_lattice.h for tests/test_lattice.py
// (the device code is the same header compiled by hipcc).
#include "../../firedancer_amd/csrc/fdgpu_lattice.h"

// which = 0: hs_split (Lehmer, the kernel's), 1: hs_split_euclid (one full step at a time)
extern "C" int hs_split_host(const uint32_t *k, uint32_t *u, uint32_t *v, uint32_t *flags, int which) {
  uint32_t kk[8];
  for (int i = 0; i < 8; i++) kk[i] = k[i];
  fdgpu::hs_split_t o;
  if (which) fdgpu::hs_split_euclid(o, kk);
  else fdgpu::hs_split(o, kk);
  for (int i = 0; i < (int)HS_LIMBS; i++) { u[i] = o.u[i]; v[i] = o.v[i]; }
  flags[0] = o.ok; flags[1] = o.u_neg; flags[2] = o.v_neg; flags[3] = o.bits;
  return 0;
}
