# cfg5 tile sweep on one MI355X: tiles x batch x inflight, step-loop tile (mux 0)
# and mux-callback tile (mux 1); output gpurun_out/$1/tile_*.jsonl
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1; mkdir -p $o
SW="${SW:-1,16384,4,0;2,16384,4,0;4,16384,4,0;8,16384,4,0;1,32768,4,0;2,32768,4,0;4,32768,4,0}"
for m in ${MUXES:-0 1}; do
  echo "[$(date +%T)] cfg1 mux=$m"
  timeout -k 10 400 python3 tools/bench_tile.py --mux $m --multi 0 --txns 2000000 --depth-lg 21 --sweep "$SW" --out $o/tile_cfg1_mux$m.jsonl > $o/tile_cfg1_mux$m.log 2>&1 || { tail $o/tile_cfg1_mux$m.log; exit 1; }
  python3 -c "
import json
for l in open('$o/tile_cfg1_mux$m.jsonl'):
    d=json.loads(l); print('mux=$m', d['tiles'], d['batch_txn_max'], d['txns_per_s'], d['wall_s'], d['producer_s'], d['batch_latency_ms'], d['counters']['published']==d['expected_published'], d['counters']['overrun'])"
done
