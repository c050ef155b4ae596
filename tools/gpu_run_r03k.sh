# round-3 call: mux-tile capacity vs slots in flight and batch size
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03k; mkdir -p $o
echo "[$(date +%T)] capacity sweep"
timeout -k 10 600 python3 tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 0 --txns 1000000 --depth-lg 21 --reps 2 \
  --producers-same-as-tiles 1 \
  --sweep "1,16384,4,-1;1,16384,8,-1;1,32768,4,-1;1,8192,8,-1;2,16384,8,-1;2,32768,4,-1;2,16384,4,-1" \
  --out $o/cap.jsonl > $o/cap.log 2>&1 || { tail $o/cap.log; exit 1; }
python3 -c "
import json
for l in open('$o/cap.jsonl'):
    d=json.loads(l); c=d['counters']
    print(' tiles', d['tiles'], 'batch', d['batch_txn_max'], 'inflight', d['inflight'], d['txns_per_s'], d['batch_latency_ms'], 'ovr', c['overrun'], 'pub_ok', c['published']==d['expected_published'], 'poll_ms', round(c['poll_ns']/1e6,1), 'submit_ms', round(c['submit_ns']/1e6,1))"
echo "[$(date +%T)] done"
