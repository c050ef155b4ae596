# Head record: the driver's round-end steps (GPU tests, smoke, default bench) in one call.
# usage: bash tools/gpu_runs/r05/gpu_r05full.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-m}; O=gpurun_out/r05_$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" $O/gpu_tests.log | head -20; tail -5 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail -20 $O/bench.err; exit 1; }
python -c "
import json
d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline']['frac'], {k: v for k, v in d.items() if k.startswith('tile_') and (k.endswith('txns_per_s') or k.endswith('sigs_per_s') or 'p99' in k or 'published_ok' in k)})
"
