# round-3 call: tile capacity sweep (prefilled links), the full bench line,
# then the 8-rank rehearsal of the driver's multi-GPU bench on this one GPU
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03f; mkdir -p $o
echo "[$(date +%T)] tile capacity sweep"
timeout -k 10 400 python3 tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 0 --txns 1000000 --depth-lg 21 \
  --producers-same-as-tiles 1 --sweep "1,16384,4,-1;2,16384,4,-1;3,16384,4,-1;4,16384,4,-1;1,8192,4,-1;2,8192,4,-1" \
  --out $o/mux_cap.jsonl > $o/mux_cap.log 2>&1 || { tail $o/mux_cap.log; exit 1; }
python3 -c "
import json
for l in open('$o/mux_cap.jsonl'):
    d=json.loads(l); c=d['counters']
    print(' tiles', d['tiles'], 'batch', d['batch_txn_max'], 'rate', d['rate_target'], d['txns_per_s'], d['batch_latency_ms'], 'ovr', c['overrun'], 'pub_ok', c['published']==d['expected_published'], 'submit_ms', round(c['submit_ns']/1e6,1), 'poll_ms', round(c['poll_ns']/1e6,1), 'wall', d['wall_s'])"
echo "[$(date +%T)] bench"
timeout -k 10 600 python3 bench.py > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
cat $o/bench.json
bash tools/gpu_rehearse8.sh r03f
