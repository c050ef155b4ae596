set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03d; mkdir -p $o
echo "[$(date +%T)] submit profile"
FDGPU_SUBMIT_PROF=1 timeout -k 10 300 python3 tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 0 --txns 1000000 --depth-lg 21 \
    --producers-same-as-tiles 1 --sweep "1,16384,4,0;1,16384,4,14000000;2,16384,4,0" --out $o/mux_prof.jsonl > $o/mux_prof.log 2>&1 || { tail $o/mux_prof.log; exit 1; }
grep -E "submit_frags_io|txns_per_s" $o/mux_prof.log | cut -c1-300
python3 -c "
import json
for l in open('$o/mux_prof.jsonl'):
    d=json.loads(l); c=d['counters']
    print(' tiles', d['tiles'], 'rate', d['rate_target'], d['txns_per_s'], d['batch_latency_ms'], 'ovr', c['overrun'], 'pub_ok', c['published']==d['expected_published'], 'batches', c['batches'], 'submit_ms', round(c['submit_ns']/1e6,1), 'poll_ms', round(c['poll_ns']/1e6,1), 'wall', d['wall_s'])"
bash tools/gpu_kernel_ab.sh r03d_ab "main tbld unroll shasm all3"
