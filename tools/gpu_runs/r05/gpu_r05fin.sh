set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05fin; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ingest.py tests/test_tile_gpu.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|assert|FAIL" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
GPU_MAX_HW_QUEUES=32 timeout -k 10 200 python -u tools/io_probe.py --npz /tmp/cfg1.npz --engines 2 --batches 300 --pair 0 --spread 0 --out $O/probe.jsonl > $O/probe.log 2>&1 || { echo PROBE_FAILED; tail $O/probe.log; exit 1; }
GPU_MAX_HW_QUEUES=32 timeout -k 10 200 python -u tools/io_probe.py --npz /tmp/cfg1.npz --engines 2 --batches 300 --pair 0 --spread 0 --out $O/probe.jsonl >> $O/probe.log 2>&1 || { echo PROBE_FAILED; tail $O/probe.log; exit 1; }
grep -o '"txns_per_s": [0-9.]*' $O/probe.jsonl
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --depth-lg-paced 14 --paced-reps 4 --pair 2 --spread 2 --wait-us 200 --reps 3 --hw-queues 32 --producers-same-as-tiles 1 --pin 1 --warm-runs 1"
for rep in 1 2; do
timeout -k 10 170 python -u tools/bench_tile.py $C --sweep "1,16384,8,-1,1;2,16384,8,-1,2;2,16384,8,24e6,4" --out $O/t$rep.jsonl > $O/t$rep.log 2>&1; rc=$?; [ $rc -le 1 ] || { echo RUN_FAILED; tail -5 $O/t$rep.log; exit 1; }
python -c "
import json
for l in open('$O/t$rep.jsonl'):
  d=json.loads(l); c=d['counters']; print(d['tiles'], d['rate_target']/1e6, round(d['txns_per_s']/1e6,2), d['batch_latency_ms'], c['overrun'], d['published_ok'])
"
done
