set -o pipefail
o=gpurun_out/g10; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 100000 --latency-batches 100 > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$o/bench.json'));print({k:d[k] for k in ('value','ms_per_step','p50_batch_latency_ms','p99_batch_latency_ms','pcie_inclusive_sigs_per_s_per_gpu','cfg3_sigs_per_s')})"
timeout -k 10 400 python -u tools/bench_tile.py --gpus 1 --txns 1000000 --depth-lg 20 --out $o/tile_sweep.jsonl \
  --sweep "1,4096,3,0;1,8192,3,0;2,8192,3,0;1,4096,3,1000000" > $o/sweep.log 2>&1 || { tail $o/sweep.log; exit 1; }
python3 -c "
import json
for l in open('$o/tile_sweep.jsonl'):
    d=json.loads(l); print(d['tiles'], d['batch_txn_max'], d['rate_target'], d['txns_per_s'], d['sigs_per_s'], d['batch_latency_ms'], d['counters']['overrun'])"
