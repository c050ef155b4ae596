set -o pipefail
o=gpurun_out/g11; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 400 python -u tools/bench_tile.py --gpus 1 --txns 1000000 --depth-lg 20 --inflight 3 --out $o/tile_sweep.jsonl \
  --sweep "1,4096,3,0;1,8192,3,0;2,4096,3,0;1,4096,3,1000000;1,4096,3,2000000" > $o/sweep.log 2>&1 || { tail $o/sweep.log; exit 1; }
python3 -c "
import json
for l in open('$o/tile_sweep.jsonl'):
    d=json.loads(l); print(d['tiles'], d['batch_txn_max'], d['rate_target'], d['txns_per_s'], d['sigs_per_s'], d['batch_latency_ms'], d['counters']['overrun'], d['counters']['published']==d['expected_published'])"
