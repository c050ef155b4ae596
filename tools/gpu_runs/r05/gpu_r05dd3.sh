# the cross-process lines with the sandboxed dedup process reading the verify tiles' out links
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05dd3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --depth-lg-paced 14 --paced-reps 4 --pair 2 --spread 2 --wait-us 200 --reps 3 --hw-queues 32 --producers-same-as-tiles 1 --pin 1 --xproc 1 --pages 4k"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_engine_proc.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for dd in 1; do
  timeout -k 10 400 python -u tools/bench_tile.py $C --dedup $dd --sweep "1,16384,8,16e6,2;2,16384,8,24e6,4;1,16384,8,-1,1;2,16384,8,-1,2" --out $O/d$dd.jsonl > $O/d$dd.log 2>&1; rc=$?; [ $rc -le 1 ] || { echo RUN_FAILED $dd rc $rc; tail -5 $O/d$dd.log; exit 1; }
  python -c "
import json
for l in open('$O/d$dd.jsonl'):
  d=json.loads(l); c=d['counters']; print('dedup $dd', d['tiles'], d['rate_target']/1e6, round(d['txns_per_s']/1e6,2), d['batch_latency_ms'], c['overrun'], c['backpressure'], d['published_ok'], json.dumps(d.get('dedup'))[:220])
"
done
