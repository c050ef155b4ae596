# round-3 call: mux-tile capacity with more signatures in flight, and a kernel trace of the two-tile run
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03l; mkdir -p $o
echo "[$(date +%T)] capacity sweep (32 hw queues)"
timeout -k 10 400 python3 tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 0 --txns 1000000 --depth-lg 21 --reps 2 \
  --producers-same-as-tiles 1 --hw-queues 32 \
  --sweep "1,8192,16,-1;2,8192,8,-1;2,8192,16,-1;2,16384,8,-1" \
  --out $o/cap.jsonl > $o/cap.log 2>&1 || { tail $o/cap.log; exit 1; }
python3 -c "
import json
for l in open('$o/cap.jsonl'):
    d=json.loads(l); c=d['counters']
    print(' tiles', d['tiles'], 'batch', d['batch_txn_max'], 'inflight', d['inflight'], d['txns_per_s'], d['batch_latency_ms'], 'ovr', c['overrun'], 'pub_ok', c['published']==d['expected_published'], 'poll_ms', round(c['poll_ns']/1e6,1), 'submit_ms', round(c['submit_ns']/1e6,1))"
echo "[$(date +%T)] kernel trace, two tiles 16384x8"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- \
  python3 tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 0 --txns 1000000 --depth-lg 21 --reps 1 \
  --producers-same-as-tiles 1 --sweep "2,16384,8,-1" --out $o/trace_run.jsonl > $o/trace.log 2>&1 || { tail $o/trace.log; exit 1; }
find $o/trace -name "*.csv" | head -20
echo "[$(date +%T)] done"
