# round-3 call: mux-tile capacity with the fused parse + expand (no scan kernel), 16 vs 32 hardware queues
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03s; mkdir -p $o
for q in 16 32; do
  echo "[$(date +%T)] capacity, $q hw queues"
  timeout -k 10 300 python3 tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 0 --txns 1000000 --depth-lg 21 --reps 2 --hw-queues $q \
    --producers-same-as-tiles 1 --sweep "1,16384,4,-1;1,16384,8,-1;2,16384,4,-1;2,16384,8,-1" --out $o/cap$q.jsonl > $o/cap$q.log 2>&1 || { tail $o/cap$q.log; exit 1; }
  python3 -c "
import json
for l in open('$o/cap$q.jsonl'):
    d=json.loads(l); c=d['counters']; b=max(1,c['batches'])
    print(' tiles', d['tiles'], 'batch', d['batch_txn_max'], 'x', d['inflight'], round(d['txns_per_s']/1e6,2), 'M', d['batch_latency_ms'], 'txn/batch', round(d['txns']/b), 'per batch ms: fill %.3f gpu %.3f publish %.3f' % (c['batch_fill_ns']/b/1e6, c['batch_gpu_ns']/b/1e6, c['publish_ns']/b/1e6), 'polls', c['polls'], 'ovr', c['overrun'], 'pub_ok', c['published']==d['expected_published'])"
done
echo "[$(date +%T)] done"
