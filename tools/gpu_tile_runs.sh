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
if [ -n "$HOSTPROF" ]; then          # host-only: T mux tiles over one prefilled link, null verifier
  python3 -c "
import sys; sys.path.insert(0,'.')
from firedancer_amd import workload
a,t,m = workload.cfg1(1000000, seed=5)
arena, offs, sizes = workload.pack_payloads(workload.payloads(a,t))
arena.tofile('/tmp/pl.bin'); offs.tofile('/tmp/pl_off.bin'); sizes.tofile('/tmp/pl_sz.bin')" || exit 1
  g++ -O2 -g -std=c++17 -I include tools/tile_prof.cpp -x c tools/null_verifier.c -o /tmp/tile_prof -L firedancer_amd \
    -l:libfd_verify_tile.so -Wl,-rpath,$PWD/firedancer_amd -lpthread -ldl -lrt || exit 1
  for T in 1 2 4; do
    TILE_PROF_TILES=$T TILE_PROF_CPU=4 TILE_PROF_OFF=1 timeout -k 10 120 /tmp/tile_prof /tmp/pl.bin /tmp/pl_off.bin \
      /tmp/pl_sz.bin ${GP:-1} 3 > $o/hostprof_T$T.txt 2>&1 || exit 1
    grep best $o/hostprof_T$T.txt | sed "s/^/ host-only $T tiles: /"
  done
fi
echo "[$(date +%T)] done"
