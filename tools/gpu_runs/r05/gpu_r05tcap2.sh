# Engine-only gathered capacity (io_probe) head vs previous kernel, two-lane kernel off / on
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05tcap2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
for pair in 0 1; do for v in "head::firedancer_amd/libfd_ed25519_gpu.so" "prev::build/prev/libfd_ed25519_gpu.so"; do
  tag=${v%%::*}; lib=${v#*::}
  FDGPU_LIB=$lib GPU_MAX_HW_QUEUES=32 timeout -k 10 200 python -u tools/io_probe.py --npz /tmp/cfg1.npz --engines 2 --batches 200 --pair $pair --spread 0 --tag ${tag}_p$pair --out $O/probe.jsonl > $O/probe_${tag}_$pair.log 2>&1 || { echo PROBE_FAILED; tail $O/probe_${tag}_$pair.log; exit 1; }
  tail -1 $O/probe_${tag}_$pair.log
done; done
