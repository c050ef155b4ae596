# round-3 call: full GPU suite, smoke, bench (tile lines at 8 in flight, 32 hardware queues)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03t; mkdir -p $o
echo "[$(date +%T)] GPU tests"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests \
  > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -1 $o/gpu_tests.log
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log | cut -c1-300
echo "[$(date +%T)] bench"
timeout -k 10 900 python3 bench.py > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$o/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'])
for k,v in d.items():
    if k.startswith('tile_') and not k.endswith('_runs'): print(' ', k, v)
for k in ('latency_ms_p50_p99_staged','latency_ms_p50_p99_registered','sync_verify_latency_us_p50_p99'):
    print(' ', k, d.get(k))"
echo "[$(date +%T)] done"
