# Mux verify tile on one MI355X: GPU tests of the tile/engine/ingest paths,
# then bench_tile sweeps of the mux tile (GPU parse vs host parse, 1-4 tiles
# over as many quic links), then the host-only cost profile (tools/tile_prof).
# usage: bash tools/gpu_tile_mux.sh <outdir> [skiptests]
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1; mkdir -p $o
if [ -z "$2" ]; then
  echo "[$(date +%T)] gpu tests (engine, tile, ingest)"
  timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_tile_gpu.py tests/test_gpu_ingest.py -x -v \
    --timeout 240 --timeout-method thread > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
  tail -1 $o/tests.log
fi
echo "[$(date +%T)] bench_tile mux cfg1"
SW="${SW:-1,16384,4,0;1,16384,4,12000000;2,16384,4,0;2,16384,4,16000000;4,16384,4,0}"
for gp in 1 0; do
  for P in ${PRODS:-same 1}; do
    timeout -k 10 400 python3 tools/bench_tile.py --mux 1 --gpu-parse $gp --multi 0 --txns 1000000 --depth-lg 21 \
      --producers-same-as-tiles $([ $P = same ] && echo 1 || echo 0) --sweep "$SW" --out $o/mux_gp${gp}_p$P.jsonl \
      > $o/mux_gp${gp}_p$P.log 2>&1 || { tail $o/mux_gp${gp}_p$P.log; exit 1; }
    python3 -c "
import json
for l in open('$o/mux_gp${gp}_p$P.jsonl'):
    d=json.loads(l); print('gp=$gp prods', d['producers'], 'tiles', d['tiles'], 'rate', d['rate_target'], d['txns_per_s'], d['batch_latency_ms'], 'pub', d['counters']['published'], d['expected_published'], 'ovr', d['counters']['overrun'], 'prod_s', d['producer_s'])"
  done
done
echo "[$(date +%T)] tile_prof (host only)"
python3 -c "
import sys; sys.path.insert(0,'.')
from firedancer_amd import workload
a,t,m = workload.cfg1(1000000, seed=5)
arena, offs, sizes = workload.pack_payloads(workload.payloads(a,t))
arena.tofile('/tmp/pl.bin'); offs.tofile('/tmp/pl_off.bin'); sizes.tofile('/tmp/pl_sz.bin')" || exit 1
g++ -O2 -g -std=c++17 -I include tools/tile_prof.cpp -x c tools/null_verifier.c -o /tmp/tile_prof -L firedancer_amd \
  -l:libfd_verify_tile.so -Wl,-rpath,$PWD/firedancer_amd -lpthread -ldl -lrt || exit 1
for gp in 1 0; do
  TILE_PROF_OFF=1 timeout -k 10 120 taskset -c 2 /tmp/tile_prof /tmp/pl.bin /tmp/pl_off.bin /tmp/pl_sz.bin $gp 5 > $o/prof_gp$gp.txt 2>&1 || exit 1
  TILE_PROF_RAW=$o/pcs_gp$gp.txt timeout -k 10 120 taskset -c 2 /tmp/tile_prof /tmp/pl.bin /tmp/pl_off.bin /tmp/pl_sz.bin $gp 3 >> $o/prof_gp$gp.txt 2>&1 || exit 1
  grep -E "^run|best" $o/prof_gp$gp.txt
done
echo "[$(date +%T)] done"
