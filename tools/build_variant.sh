#!/bin/bash
# Build an A/B variant of the engine library into build/<name>/libfd_ed25519_gpu.so
# usage: tools/build_variant.sh <name> [-DMACRO=V ...]   (load it with FDGPU_LIB=...)
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/build/$name; mkdir -p "$out"
cd "$root/firedancer_amd/csrc"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $*"
/opt/rocm/bin/hipcc $F -c fdgpu_kernels.hip -o "$out/k.o" -Rpass-analysis=kernel-resource-usage 2>&1 \
  | grep -A12 "dsm_kernel\|prep_kernel" | grep -E "Name|VGPRs|Occupancy" | sed 's/.*remark: *//' || true
/opt/rocm/bin/hipcc $F -x hip -c fdgpu_engine.cpp -o "$out/e.o"
/opt/rocm/bin/hipcc $F -shared -o "$out/libfd_ed25519_gpu.so" "$out/k.o" "$out/e.o"
echo "built $out/libfd_ed25519_gpu.so"
