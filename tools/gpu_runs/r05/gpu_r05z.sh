set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05z; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_engine.py tests/test_abi.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|assert|FAIL" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in "big::X=1" "off::FDGPU_BIG_STREAMS=0" "big2::X=1"; do
  tag=${v%%::*}; envs=${v#*::}
  timeout -k 10 300 env $envs python -u tools/host_fed_probe.py --ring 2,3,4 --feed registered,staged --steps 12 --reps 1 > $O/hf_$tag.log 2>&1 || { echo HF_FAILED $tag; tail -20 $O/hf_$tag.log; exit 1; }
  grep '^{' $O/hf_$tag.log | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); print('$tag', d['feed'], d['ring'], round(d['sigs_per_s']/1e6,1), d['ms_per_batch'], d['codes_equal'])
"
done
