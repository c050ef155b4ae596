set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05hf; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_engine.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|assert|FAIL" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools/host_fed_probe.py --ring 3 --feed registered,staged --steps 12 --reps 2 > $O/hf_$rep.log 2>&1 || { echo HF_FAILED; tail -20 $O/hf_$rep.log; exit 1; }
  grep '^{' $O/hf_$rep.log | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); print(d['feed'], d['ring'], round(d['sigs_per_s']/1e6,1), d['ms_per_batch'], d['submit_stage_expand_enqueue_ms'], d['codes_equal'])
"
done
