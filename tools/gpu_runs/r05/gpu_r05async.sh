set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05async; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --depth-lg-paced 14 --paced-reps 4 --pair 2 --spread 2 --wait-us 200 --reps 3 --hw-queues 32 --producers-same-as-tiles 1 --pin 1 --warm-runs 1"
for rep in 1 2; do for v in "sync::FDT_ASYNC_SUBMIT=0" "async::FDT_ASYNC_SUBMIT=1"; do
  tag=${v%%::*}; envs=${v#*::}
  timeout -k 10 170 env $envs python -u tools/bench_tile.py $C --sweep "1,16384,8,-1,1;2,16384,8,-1,2;2,16384,8,24e6,4;1,16384,8,36e6,3" --out $O/${tag}_$rep.jsonl > $O/${tag}_$rep.log 2>&1; rc=$?; [ $rc -le 1 ] || { echo RUN_FAILED $tag rc $rc; tail -5 $O/${tag}_$rep.log; exit 1; }
  python -c "
import json
for l in open('$O/${tag}_$rep.jsonl'):
  d=json.loads(l); c=d['counters']; print('$tag', d['tiles'], d['rate_target']/1e6, round(d['txns_per_s']/1e6,2), d['batch_latency_ms'], 'ovr', c['overrun'], 'sub_us', round(c['submit_ns']/c['batches']/1e3,1), d['published_ok'])
"
done; done
