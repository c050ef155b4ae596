set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ingest.py tests/test_tile_gpu.py tests/test_engine_proc.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|assert|FAIL" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
timeout -k 10 200 python tools/make_tile_npz.py --multi 1 --out /tmp/cfg3.npz >> $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --depth-lg 21 --depth-lg-paced 14 --paced-reps 4 --pair 2 --spread 2 --wait-us 200 --reps 3 --hw-queues 32 --producers-same-as-tiles 1"
timeout -k 10 170 python -u tools/bench_tile.py $C --payload-npz /tmp/cfg1.npz --sweep "1,16384,8,12e6,2;2,16384,8,24e6,4;1,16384,8,-1,1;2,16384,8,-1,2;2,16384,10,-1,2;2,16384,6,-1,2" --out $O/cfg1.jsonl > $O/cfg1.log 2>&1 || { echo RUN_FAILED cfg1; tail -5 $O/cfg1.log; exit 1; }
timeout -k 10 170 python -u tools/bench_tile.py $C --multi 1 --batch-sig-max 24576 --payload-npz /tmp/cfg3.npz --sweep "1,16384,8,-1,1,24576;2,16384,8,-1,2,16384;2,16384,8,-1,2,24576" --out $O/cfg3.jsonl > $O/cfg3.log 2>&1 || { echo RUN_FAILED cfg3; tail -5 $O/cfg3.log; exit 1; }
python -c "
import json
for t in ('cfg1','cfg3'):
  for l in open('$O/'+t+'.jsonl'):
    d=json.loads(l); print(t, d['tiles'], d['inflight'], d.get('batch_sig_max'), d['rate_target'], round(d['txns_per_s']/1e6,2), round(d['sigs_per_s']/1e6,2), d['batch_latency_ms'], d['published_ok'])
"
