# Registered feed after the slack memset kernel became a copy: tests + probe A/B + trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05reg3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_engine.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u tools/host_fed_probe.py --ring 3 --feed registered,staged --steps 12 --reps 2 > $O/probe.log 2>&1 || { echo PROBE_FAILED; tail $O/probe.log; exit 1; }
grep feed $O/probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o run -- python3 -u tools/host_fed_probe.py --ring 3 --feed registered --steps 12 > $O/tr.log 2>&1 || { echo TRACE_FAILED; tail $O/tr.log; exit 1; }
timeout -k 10 600 python -u bench.py --steps 10 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail $O/bench.err; exit 1; }
python -c "
import json
d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], {k: v for k, v in d.items() if k.startswith('host_fed') and ('per_s' in k or 'vs_' in k or 'equal' in k)})
"
