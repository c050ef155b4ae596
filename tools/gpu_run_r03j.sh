# round-3 call: smoke, tile capacity x3, host-only tile profile, full bench
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03j; mkdir -p $o
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log | cut -c1-400
echo "[$(date +%T)] tile capacity x3"
timeout -k 10 500 python3 tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 0 --txns 1000000 --depth-lg 21 --reps 3 \
  --producers-same-as-tiles 1 --sweep "1,16384,4,-1;2,16384,4,-1;2,16384,4,30000000" \
  --out $o/cap.jsonl > $o/cap.log 2>&1 || { tail $o/cap.log; exit 1; }
python3 -c "
import json
for l in open('$o/cap.jsonl'):
    d=json.loads(l); c=d['counters']
    print(' tiles', d['tiles'], 'rate', d['rate_target'], d['txns_per_s'], d['batch_latency_ms'], 'ovr', c['overrun'], 'pub_ok', c['published']==d['expected_published'])"
echo "[$(date +%T)] host-only tile profile"
python3 -c "
import sys; sys.path.insert(0,'.')
from firedancer_amd import workload
a,t,m = workload.cfg1(1000000, seed=5)
arena, offs, sizes = workload.pack_payloads(workload.payloads(a,t))
arena.tofile('/tmp/pl.bin'); offs.tofile('/tmp/pl_off.bin'); sizes.tofile('/tmp/pl_sz.bin')" || exit 1
g++ -O2 -g -std=c++17 -I include tools/tile_prof.cpp -x c tools/null_verifier.c -o /tmp/tile_prof -L firedancer_amd \
  -l:libfd_verify_tile.so -Wl,-rpath,$PWD/firedancer_amd -lpthread -ldl -lrt 2>/dev/null || exit 1
for T in 1 2; do
  TILE_PROF_TILES=$T TILE_PROF_CPU=4 TILE_PROF_OFF=1 timeout -k 10 120 /tmp/tile_prof /tmp/pl.bin /tmp/pl_off.bin \
    /tmp/pl_sz.bin 2 3 > $o/hostprof_T$T.txt 2>&1 || exit 1
  grep best $o/hostprof_T$T.txt | sed "s/^/ host-only $T tiles: /"
done
echo "[$(date +%T)] bench"
timeout -k 10 600 python3 bench.py > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
python3 -c "
import json
d=json.load(open('$o/bench.json'))
print({k: v for k, v in d.items() if k.startswith(('value','ms_per','p50','p99','latency_split','submit_parts','tile_mux'))})"
echo "[$(date +%T)] done"
