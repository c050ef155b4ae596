# round-3 call: per-batch fill / GPU / publish time of the mux tile, one vs two tiles
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03o; mkdir -p $o
echo "[$(date +%T)] capacity"
timeout -k 10 300 python3 tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 0 --txns 1000000 --depth-lg 21 --reps 2 \
  --producers-same-as-tiles 1 --sweep "1,16384,4,-1;2,16384,4,-1;2,16384,8,-1;2,32768,4,-1" --out $o/cap.jsonl > $o/cap.log 2>&1 || { tail $o/cap.log; exit 1; }
python3 -c "
import json
for l in open('$o/cap.jsonl'):
    d=json.loads(l); c=d['counters']; b=max(1,c['batches'])
    print(' tiles', d['tiles'], 'batch', d['batch_txn_max'], 'x', d['inflight'], round(d['txns_per_s']/1e6,2), 'M', d['batch_latency_ms'], 'txn/batch', round(d['txns']/b), 'per batch ms: fill %.3f gpu %.3f publish %.3f' % (c['batch_fill_ns']/b/1e6, c['batch_gpu_ns']/b/1e6, c['publish_ns']/b/1e6), 'polls', c['polls'], 'poll_ms', round(c['poll_ns']/1e6,1), 'submit_ms', round(c['submit_ns']/1e6,1), 'wall_ms', round(d['wall_s']*1e3,1))"
echo "[$(date +%T)] done"
