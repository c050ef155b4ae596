# Shared identity table entry (2880-B workspace per signature): GPU parity tests + timing A/B vs the previous head
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05id; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_engine.py tests/test_gpu_parity_scale.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do for v in "prev::build/prev/libfd_ed25519_gpu.so" "ident::firedancer_amd/libfd_ed25519_gpu.so"; do
  tag=${v%%::*}; lib=${v#*::}
  FDGPU_LIB=$lib timeout -k 10 120 python3 bench.py --no-extras --steps 30 --warmup 5 > $O/time_${tag}_$i.json 2>$O/time_${tag}_$i.err || { echo TIME_FAILED $tag; tail $O/time_${tag}_$i.err; exit 1; }
  python3 -c "
import json
b=json.loads(open('$O/time_${tag}_$i.json').read().strip().splitlines()[-1]); print('$tag', $i, b['value'], b['ms_per_step'], b.get('parity_mismatches'))"
done; done
