set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|error" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail -30 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline']['frac'], d['ms_per_step'])
for k,v in d.items():
  if (k.startswith('host_fed') and 'per_s' in k) or (k.startswith('tile_') and ('txns_per_s' in k or 'p50' in k or 'sigs_per_s' in k) and 'runs' not in k) or 'latency' in k: print(k, v)
"
