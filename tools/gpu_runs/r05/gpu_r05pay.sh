# Which side should pay for the out frags' payload bytes:
# the device writing them back over PCIe (gather, the default), or the tile core
# copying them (mode 1: the tile copies each payload into its out frag, the GPU
# parses and verifies the copies) -- and a diagnostic build that skips the
# payload's write-back (wrong output) to price those PCIe writes alone.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05pay; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --payload-npz /tmp/cfg1.npz --depth-lg 21 --depth-lg-paced 14 --paced-reps 4 --pair 2 --spread 2 --wait-us 200 --reps 4 --hw-queues 32 --producers-same-as-tiles 1 --pin 1"
for rep in 1 2; do
for v in "gather::.::2" "copy::.::1" "nopay::build/ab/nopay::2"; do
  tag=${v%%::*}; rest=${v#*::}; dir=${rest%%::*}; gp=${rest#*::}
  for sw in "1,16384,8,-1,1" "2,16384,8,-1,2"; do
    ( cd $dir && timeout -k 10 170 python -u tools/bench_tile.py $C --gpu-parse $gp --sweep "$sw" --out $O/${tag}_$rep.jsonl >> $O/${tag}.log 2>&1 ) || { echo RUN_FAILED $tag; tail -5 $O/${tag}.log; exit 1; }
  done
done; done
for tag in gather copy nopay; do grep '^{"metric"' $O/$tag.log | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); c=d['counters']; print('$tag', d['tiles'], round(d['txns_per_s']/1e6,2), d['batch_latency_ms'], d['published_ok'])
"; done
