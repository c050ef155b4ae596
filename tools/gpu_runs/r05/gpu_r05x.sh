set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05x; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --depth-lg-paced 14 --paced-reps 4 --pair 2 --spread 2 --wait-us 200 --reps 3 --hw-queues 32 --producers-same-as-tiles 1 --pin 1"
for sw in "2,16384,8,-1,2" "2,16384,10,-1,2" "2,24576,8,-1,2" "2,12288,10,-1,2" "3,16384,6,-1,3" "2,16384,9,-1,2" "2,20480,8,-1,2"; do
  timeout -k 10 170 python -u tools/bench_tile.py $C --sweep "$sw" --out $O/x.jsonl >> $O/x.log 2>&1 || { echo RUN_FAILED $sw; tail -5 $O/x.log; exit 1; }
done
grep '^{"metric"' $O/x.log | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); print(d['tiles'], d['batch_txn_max'], d['inflight'], round(d['txns_per_s']/1e6,2), d['batch_latency_ms'], d['published_ok'])
"
