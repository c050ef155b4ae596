# round-3 call: gather-path GPU tests (in-place writes), tile sweep with the
# submit profile, then the kernel A/B
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03e; mkdir -p $o
echo "[$(date +%T)] gpu tests (ingest, tile)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ingest.py tests/test_tile_gpu.py -x -v --timeout 240 \
  --timeout-method thread > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
echo "[$(date +%T)] tile sweep (gather, in-place writes)"
FDGPU_SUBMIT_PROF=1 timeout -k 10 400 python3 tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 0 --txns 1000000 \
  --depth-lg 21 --producers-same-as-tiles 1 \
  --sweep "1,16384,4,0;1,16384,4,12000000;1,16384,4,16000000;2,16384,4,0;2,16384,4,16000000;2,16384,4,24000000;4,16384,4,0" \
  --out $o/mux_gp2.jsonl > $o/mux_gp2.log 2>&1 || { tail $o/mux_gp2.log; exit 1; }
grep -E "submit_frags_io" $o/mux_gp2.log | tail -3
python3 -c "
import json
for l in open('$o/mux_gp2.jsonl'):
    d=json.loads(l); c=d['counters']
    print(' tiles', d['tiles'], 'rate', d['rate_target'], d['txns_per_s'], d['batch_latency_ms'], 'ovr', c['overrun'], 'pub_ok', c['published']==d['expected_published'], 'batches', c['batches'], 'submit_ms', round(c['submit_ns']/1e6,1), 'poll_ms', round(c['poll_ns']/1e6,1), 'wall', d['wall_s'])"
bash tools/gpu_kernel_ab.sh r03e_ab "main tbld unroll shasm all3"
