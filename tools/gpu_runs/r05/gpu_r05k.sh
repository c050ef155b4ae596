set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05k; mkdir -p $O
export TMPDIR=/tmp FDGPU_IO_DMA=0
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --depth-lg-paced 14 --paced-reps 4 --pair 2 --spread 2 --wait-us 200 --reps 3 --hw-queues 32 --producers-same-as-tiles 1"
S="1,16384,8,-1,1;2,16384,8,-1,2"
for rep in 1 2; do
for tag in old head wt; do
  ( cd build/ab/$tag && timeout -k 10 300 python -u tools/bench_tile.py $C --sweep "$S" --out $O/${tag}_$rep.jsonl > $O/${tag}_$rep.log 2>&1 ) || { echo RUN_FAILED $tag; tail -5 $O/${tag}_$rep.log; exit 1; }
  python -c "
import json
for l in open('$O/${tag}_$rep.jsonl'):
  d=json.loads(l); c=d['counters']; print('$tag', d['tiles'], d['rate_target'], round(d['txns_per_s']/1e6,2), d['batch_latency_ms'], d['published_ok'])
"
done; done
