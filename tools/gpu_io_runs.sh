set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03c; mkdir -p $o
echo "[$(date +%T)] gpu tests (ingest io, tile)"
timeout -k 10 500 python -u -m pytest tests/test_gpu_ingest.py tests/test_tile_gpu.py -x -v --timeout 240 --timeout-method thread > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for gp in 2 1; do
  echo "[$(date +%T)] bench_tile gp=$gp"
  timeout -k 10 400 python3 tools/bench_tile.py --mux 1 --gpu-parse $gp --multi 0 --txns 1000000 --depth-lg 21 \
    --producers-same-as-tiles 1 --sweep "1,16384,4,0;1,16384,4,12000000;2,16384,4,0;2,16384,4,16000000;4,16384,4,0;4,16384,4,24000000" --out $o/mux_gp$gp.jsonl > $o/mux_gp$gp.log 2>&1 || { tail $o/mux_gp$gp.log; exit 1; }
  python3 -c "
import json
for l in open('$o/mux_gp$gp.jsonl'):
    d=json.loads(l); c=d['counters']
    print(' tiles', d['tiles'], 'rate', d['rate_target'], d['txns_per_s'], d['batch_latency_ms'], 'ovr', c['overrun'], 'pub_ok', c['published']==d['expected_published'], 'submit_ms', round(c['submit_ns']/1e6,1), 'poll_ms', round(c['poll_ns']/1e6,1), 'wall', d['wall_s'])"
done
echo "[$(date +%T)] done"
