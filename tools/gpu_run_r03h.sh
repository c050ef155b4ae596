# round-3 call: mux-tile capacity, three runs each (16 HIP queues, mcache
# prefetch), then the full bench line (latency loop pinned)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03h; mkdir -p $o
echo "[$(date +%T)] tile capacity x3"
timeout -k 10 500 python3 tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 0 --txns 1000000 --depth-lg 21 --reps 3 \
  --producers-same-as-tiles 1 --sweep "1,16384,4,-1;2,16384,4,-1;4,16384,4,-1;2,16384,4,30000000" \
  --out $o/cap.jsonl > $o/cap.log 2>&1 || { tail $o/cap.log; exit 1; }
python3 -c "
import json
for l in open('$o/cap.jsonl'):
    d=json.loads(l); c=d['counters']
    print(' tiles', d['tiles'], 'rate', d['rate_target'], d['txns_per_s'], d['batch_latency_ms'], 'ovr', c['overrun'], 'pub_ok', c['published']==d['expected_published'], 'submit_ms', round(c['submit_ns']/1e6,1), 'poll_ms', round(c['poll_ns']/1e6,1))"
echo "[$(date +%T)] bench"
timeout -k 10 600 python3 bench.py > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
python3 -c "
import json
d=json.load(open('$o/bench.json'))
print({k: v for k, v in d.items() if k.startswith(('value','ms_per','p50','p99','latency_split','tile_mux'))})"
echo "[$(date +%T)] done"
