# round-3 call: gather path with no upload copy and no memset (the gather reads the records in place and clears the verify counter)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03n; mkdir -p $o
echo "[$(date +%T)] gather-path GPU tests"
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_ingest.py tests/test_tile_gpu.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
echo "[$(date +%T)] capacity"
FDGPU_SUBMIT_PROF=1 timeout -k 10 300 python3 tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 0 --txns 1000000 --depth-lg 21 --reps 2 \
  --producers-same-as-tiles 1 --sweep "1,16384,4,-1;1,8192,8,-1;2,16384,4,-1;2,8192,8,-1" --out $o/cap.jsonl > $o/cap.log 2>&1 || { tail $o/cap.log; exit 1; }
grep "submit_frags_io" $o/cap.log | sort | uniq -c | head; python3 -c "
import json
for l in open('$o/cap.jsonl'):
    d=json.loads(l); c=d['counters']
    print(' tiles', d['tiles'], 'batch', d['batch_txn_max'], 'inflight', d['inflight'], d['txns_per_s'], d['batch_latency_ms'], 'ovr', c['overrun'], 'pub_ok', c['published']==d['expected_published'], 'poll_ms', round(c['poll_ns']/1e6,1), 'submit_ms', round(c['submit_ns']/1e6,1), 'polls', c.get('polls'), 'poll_done_ms', round(c.get('poll_done_ns',0)/1e6,1), 'publish_ms', round(c.get('publish_ns',0)/1e6,1), 'wall_ms', round(d['wall_s']*1e3,1))"
echo "[$(date +%T)] done"
