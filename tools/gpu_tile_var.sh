# Tile throughput variance study on one MI355X box: per-CPU speed, the
# host-only mux-tile cost (pinned), and repeated bench_tile runs of the mux
# tile over batch wait / in-flight depth / CPU placement.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 120 python3 tools/cpu_probe.py 64 > $o/cpu_probe.json || exit 1
cat $o/cpu_probe.json
python3 -c "
import sys; sys.path.insert(0,'.')
from firedancer_amd import workload
a,t,m = workload.cfg1(1000000, seed=5)
arena, offs, sizes = workload.pack_payloads(workload.payloads(a,t))
arena.tofile('/tmp/pl.bin'); offs.tofile('/tmp/pl_off.bin'); sizes.tofile('/tmp/pl_sz.bin')" || exit 1
g++ -O2 -g -std=c++17 -I include tools/tile_prof.cpp -x c tools/null_verifier.c -o /tmp/tile_prof -L firedancer_amd \
  -l:libfd_verify_tile.so -Wl,-rpath,$PWD/firedancer_amd -lpthread -ldl -lrt || exit 1
for gp in 1 0; do
  TILE_PROF_CPU=${PCPU:-5} TILE_PROF_OFF=1 timeout -k 10 120 /tmp/tile_prof /tmp/pl.bin /tmp/pl_off.bin /tmp/pl_sz.bin $gp 5 > $o/prof_gp$gp.txt 2>&1 || exit 1
  TILE_PROF_CPU=${PCPU:-5} TILE_PROF_RAW=$o/pcs_gp$gp.txt timeout -k 10 120 /tmp/tile_prof /tmp/pl.bin /tmp/pl_off.bin /tmp/pl_sz.bin $gp 3 >> $o/prof_gp$gp.txt 2>&1 || exit 1
  grep -E "^run|best" $o/prof_gp$gp.txt
done
for cfg in "200 4 2" "1000 4 2" "500 8 2"; do
  set -- $cfg
  echo "[$(date +%T)] wait_us=$1 inflight=$2 cpu_offset=$3"
  timeout -k 10 400 python3 tools/bench_tile.py --mux 1 --gpu-parse 1 --multi 0 --txns 1000000 --depth-lg 21 \
    --wait-us $1 --cpu-offset $3 --reps 3 --sweep "1,16384,$2,0;1,16384,$2,12000000;2,16384,$2,0" --producers-same-as-tiles 1 \
    --out $o/var_$1_$2_$3.jsonl > $o/var_$1_$2_$3.log 2>&1 || { tail $o/var_$1_$2_$3.log; exit 1; }
  python3 -c "
import json
for l in open('$o/var_$1_$2_$3.jsonl'):
    d=json.loads(l); print(' tiles', d['tiles'], 'rate', d['rate_target'], d['txns_per_s'], d['batch_latency_ms'], 'ovr', d['counters']['overrun'], 'prod_s', d['producer_s'], 'cpus', d['cpus'])"
done
echo "[$(date +%T)] done"
