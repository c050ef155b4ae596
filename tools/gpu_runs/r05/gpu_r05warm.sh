set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05warm; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --depth-lg-paced 14 --paced-reps 4 --pair 2 --spread 2 --wait-us 200 --reps 3 --hw-queues 32 --producers-same-as-tiles 1 --pin 1"
for w in 1 0 1 0; do
  timeout -k 10 170 python -u tools/bench_tile.py $C --warm-runs $w --sweep "2,16384,8,-1,2" --out $O/x.jsonl > $O/w$w.log 2>&1; rc=$?; [ $rc -le 1 ] || { echo RUN_FAILED; tail -5 $O/w$w.log; exit 1; }
  grep '^{"metric"' $O/w$w.log | python -c "
import json,sys
print('warm $w', [round(json.loads(l)['txns_per_s']/1e6,1) for l in sys.stdin])
"
  timeout -k 10 170 python -u tools/bench_tile.py $C --warm-runs $w --sweep "1,16384,8,24e6,2" --out $O/y.jsonl > $O/v$w.log 2>&1; rc=$?; [ $rc -le 1 ] || { echo RUN_FAILED; tail -5 $O/v$w.log; exit 1; }
  grep '^{"metric"' $O/v$w.log | python -c "
import json,sys
print('warm $w paced24', [(round(json.loads(l)['txns_per_s']/1e6,1), json.loads(l)['counters']['overrun'], json.loads(l)['counters']['stall_max_ns']) for l in sys.stdin])
"
done
