# Decoded R no longer parked (full path compares with the -R table): GPU parity + A/B vs the previous head
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05park; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_engine.py tests/test_gpu_keycache.py tests/test_gpu_parity_scale.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do for v in "prev::build/ident/libfd_ed25519_gpu.so" "park::firedancer_amd/libfd_ed25519_gpu.so"; do
  tag=${v%%::*}; lib=${v#*::}
  FDGPU_LIB=$lib timeout -k 10 120 python3 bench.py --no-extras --steps 30 --warmup 5 > $O/time_${tag}_$i.json 2>$O/time_${tag}_$i.err || { echo TIME_FAILED $tag; tail $O/time_${tag}_$i.err; exit 1; }
  python3 -c "
import json
b=json.loads(open('$O/time_${tag}_$i.json').read().strip().splitlines()[-1]); print('$tag', $i, b['value'], b['ms_per_step'], b.get('parity_mismatches'))"
done; done
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; exit 1; }
for v in "prev::build/ident/libfd_ed25519_gpu.so" "park::firedancer_amd/libfd_ed25519_gpu.so" "prev::build/ident/libfd_ed25519_gpu.so" "park::firedancer_amd/libfd_ed25519_gpu.so"; do
  tag=${v%%::*}; lib=${v#*::}
  FDGPU_LIB=$lib GPU_MAX_HW_QUEUES=32 timeout -k 10 200 python -u tools/io_probe.py --npz /tmp/cfg1.npz --engines 2 --batches 600 --pair 1 --spread 0 --tag ${tag}_pair --out $O/probe.jsonl > $O/probe.log 2>&1 || { echo PROBE_FAILED; tail $O/probe.log; exit 1; }
  tail -1 $O/probe.jsonl | cut -c1-160
done
