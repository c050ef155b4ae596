# round-3 call: batch-latency tails vs the submitting thread's CPU; tile capacity vs slots in flight
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03w; mkdir -p $o
echo "[$(date +%T)] latency vs pinned CPU"
timeout -k 10 300 python3 tools/lat_probe.py --pins "0,1,5,-,0" --batches 1000 > $o/lat.jsonl 2> $o/lat.err || { tail $o/lat.err; exit 1; }
cat $o/lat.jsonl
echo "[$(date +%T)] tile capacity vs slots in flight"
timeout -k 10 300 python3 tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 0 --txns 1000000 --depth-lg 21 --reps 2 \
  --producers-same-as-tiles 1 --sweep "1,16384,8,-1;1,16384,16,-1;2,16384,8,-1;2,16384,12,-1;2,16384,16,-1" --out $o/cap.jsonl > $o/cap.log 2>&1 || { tail $o/cap.log; exit 1; }
python3 -c "
import json
for l in open('$o/cap.jsonl'):
    d=json.loads(l); c=d['counters']; b=max(1,c['batches'])
    print(' tiles', d['tiles'], 'x', d['inflight'], round(d['txns_per_s']/1e6,2), 'M', d['batch_latency_ms'], 'txn/batch', round(d['txns']/b), 'gpu ms %.3f' % (c['batch_gpu_ns']/b/1e6), 'ovr', c['overrun'], 'pub_ok', c['published']==d['expected_published'])"
echo "[$(date +%T)] done"
