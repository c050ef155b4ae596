# round-3 call: where fdgpu_submit_frags_io's host time goes, one tile vs two;
# then 8 K-txn batches x 8 slots, 16 vs 32 hardware queues, 3 reps each
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03m; mkdir -p $o
summ() {
  python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); c=d['counters']
    print(' tiles', d['tiles'], 'batch', d['batch_txn_max'], 'inflight', d['inflight'], d['txns_per_s'], d['batch_latency_ms'], 'batches', c.get('batches'), 'ovr', c['overrun'], 'pub_ok', c['published']==d['expected_published'], 'poll_ms', round(c['poll_ns']/1e6,1), 'submit_ms', round(c['submit_ns']/1e6,1))" $1
}
echo "[$(date +%T)] gather-path GPU tests"
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_ingest.py tests/test_tile_gpu.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for t in 1 2; do
  echo "[$(date +%T)] submit profile, tiles $t"
  FDGPU_SUBMIT_PROF=1 timeout -k 10 200 python3 tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 0 --txns 1000000 --depth-lg 21 --reps 1 \
    --producers-same-as-tiles 1 --sweep "$t,16384,4,-1" --out $o/prof$t.jsonl > $o/prof$t.log 2>&1 || { tail $o/prof$t.log; exit 1; }
  grep -i "submit" $o/prof$t.log | tail -3
  summ $o/prof$t.jsonl
done
for q in 16 32; do
  echo "[$(date +%T)] 8K x 8, $q hw queues"
  timeout -k 10 300 python3 tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 0 --txns 1000000 --depth-lg 21 --reps 3 \
    --producers-same-as-tiles 1 --hw-queues $q --sweep "1,8192,8,-1;2,8192,8,-1" --out $o/q$q.jsonl > $o/q$q.log 2>&1 || { tail $o/q$q.log; exit 1; }
  summ $o/q$q.jsonl
done
echo "[$(date +%T)] done"
