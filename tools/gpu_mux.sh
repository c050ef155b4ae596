# vmux GPU tests + end-to-end tile throughput (step-loop tile vs mux-callback tile)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1; mkdir -p $o
echo "[$(date +%T)] tile gpu tests"
[ -n "$SKIPTEST" ] || timeout -k 10 300 python -u -m pytest tests/test_tile_gpu.py -x -v --timeout 240 --timeout-method thread > $o/tile_tests.log 2>&1 || { tail -30 $o/tile_tests.log; exit 1; }
tail -1 $o/tile_tests.log
for m in 0 1; do
  echo "[$(date +%T)] bench_tile mux=$m cfg1"
  timeout -k 10 300 python3 tools/bench_tile.py --mux $m --multi 0 --txns 1000000 --depth-lg 20 --sweep "1,4096,3,0;2,4096,3,0;4,4096,3,0" --out $o/tile_cfg1_mux$m.jsonl > $o/tile_cfg1_mux$m.log 2>&1 || { tail $o/tile_cfg1_mux$m.log; exit 1; }
  python3 -c "
import json
for l in open('$o/tile_cfg1_mux$m.jsonl'):
    d=json.loads(l); print('mux=$m', d['tiles'], d['txns_per_s'], d['sigs_per_s'], d['batch_latency_ms'], d['counters']['published'], d['expected_published'], d['counters']['overrun'])"
done
echo "[$(date +%T)] bench_tile mux=1 cfg3"
timeout -k 10 300 python3 tools/bench_tile.py --mux 1 --multi 1 --txns 300000 --depth-lg 20 --sweep "1,4096,3,0;2,4096,3,0;4,4096,3,0" --out $o/tile_cfg3_mux1.jsonl > $o/tile_cfg3_mux1.log 2>&1 || { tail $o/tile_cfg3_mux1.log; exit 1; }
python3 -c "
import json
for l in open('$o/tile_cfg3_mux1.jsonl'):
    d=json.loads(l); print('cfg3 mux=1', d['tiles'], d['txns_per_s'], d['sigs_per_s'], d['batch_latency_ms'], d['counters']['published'], d['expected_published'], d['counters']['overrun'])"
