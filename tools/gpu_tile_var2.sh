# Tile sweep with more HIP hardware queues (GPU_MAX_HW_QUEUES) so every
# in-flight batch of every tile's engine has a queue of its own.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1; mkdir -p $o
python3 -c "
import sys; sys.path.insert(0,'.')
from firedancer_amd import workload
a,t,m = workload.cfg1(1000000, seed=5)
arena, offs, sizes = workload.pack_payloads(workload.payloads(a,t))
arena.tofile('/tmp/pl.bin'); offs.tofile('/tmp/pl_off.bin'); sizes.tofile('/tmp/pl_sz.bin')" || exit 1
g++ -O2 -g -std=c++17 -I include tools/tile_prof.cpp -x c tools/null_verifier.c -o /tmp/tile_prof -L firedancer_amd \
  -l:libfd_verify_tile.so -Wl,-rpath,$PWD/firedancer_amd -lpthread -ldl -lrt || exit 1
TILE_PROF_CPU=5 TILE_PROF_OFF=1 timeout -k 10 120 /tmp/tile_prof /tmp/pl.bin /tmp/pl_off.bin /tmp/pl_sz.bin 1 5 > $o/prof_gp1.txt 2>&1 || exit 1
TILE_PROF_CPU=5 TILE_PROF_RAW=$o/pcs_gp1.txt timeout -k 10 120 /tmp/tile_prof /tmp/pl.bin /tmp/pl_off.bin /tmp/pl_sz.bin 1 3 >> $o/prof_gp1.txt 2>&1 || exit 1
grep -E "^run|best" $o/prof_gp1.txt
for cfg in "${CFGS[@]:-1000 4 2 16 1000 8 2 16 500 8 2 16}"; do :; done
run() {  # wait inflight cpu_offset hwq
  echo "[$(date +%T)] wait_us=$1 inflight=$2 cpu_offset=$3 GPU_MAX_HW_QUEUES=$4"
  GPU_MAX_HW_QUEUES=$4 timeout -k 10 400 python3 tools/bench_tile.py --mux 1 --gpu-parse 1 --multi 0 --txns 1000000 --depth-lg 21 \
    --wait-us $1 --cpu-offset $3 --reps 2 --sweep "1,16384,$2,0;1,16384,$2,12000000;2,16384,$2,0;2,16384,$2,16000000;4,16384,$2,0" \
    --producers-same-as-tiles 1 --out $o/var_$1_$2_$3_$4.jsonl > $o/var_$1_$2_$3_$4.log 2>&1 || { tail $o/var_$1_$2_$3_$4.log; exit 1; }
  python3 -c "
import json
for l in open('$o/var_$1_$2_$3_$4.jsonl'):
    d=json.loads(l); print(' tiles', d['tiles'], 'rate', d['rate_target'], d['txns_per_s'], d['batch_latency_ms'], 'ovr', d['counters']['overrun'], 'pub_ok', d['counters']['published']==d['expected_published'], 'prod_s', d['producer_s'])"
}
run 1000 4 2 16 && run 1000 8 2 16 && run 500 8 2 16 && run 1000 4 2 4
echo "[$(date +%T)] done"
