# bench_tile runs of the mux tile (GPU parse) on one MI355X.
# usage: RUNS="wait inflight cpu_off hwq sweep;..." bash tools/gpu_tile_runs.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1; mkdir -p $o
IFS=';' read -ra R <<< "${RUNS:-1000 4 2 16 1,16384,4,0:2,16384,4,0}"
for r in "${R[@]}"; do
  set -- $r
  sw=${5//:/;}
  tag=$(echo "$r" | tr ' ,:' '___')
  echo "[$(date +%T)] wait_us=$1 inflight=$2 cpu_offset=$3 GPU_MAX_HW_QUEUES=$4 sweep=$sw"
  GPU_MAX_HW_QUEUES=$4 timeout -k 10 400 python3 tools/bench_tile.py --mux 1 --gpu-parse ${GP:-1} --multi ${MULTI:-0} \
    --txns ${TXNS:-1000000} --depth-lg 21 --wait-us $1 --cpu-offset $3 --reps ${REPS:-2} --sweep "$sw" \
    --producers-same-as-tiles 1 --out gpurun_out/$tag.jsonl > gpurun_out/$tag.log 2>&1 || { tail gpurun_out/$tag.log; exit 1; }
  mv gpurun_out/$tag.jsonl gpurun_out/$tag.log $o/
  python3 -c "
import json
for l in open('$o/$tag.jsonl'):
    d=json.loads(l); c=d['counters']
    print(' tiles', d['tiles'], 'rate', d['rate_target'], d['txns_per_s'], d['batch_latency_ms'], 'ovr', c['overrun'], 'pub_ok', c['published']==d['expected_published'], 'batches', c['batches'], 'submit_ms', round(c['submit_ns']/1e6,1), 'poll_ms', round(c['poll_ns']/1e6,1), 'wall_s', d['wall_s'])"
done
echo "[$(date +%T)] done"
