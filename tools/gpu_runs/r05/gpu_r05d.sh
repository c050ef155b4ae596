set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --pair 2 --spread 2 --wait-us 200 --reps 3 --hw-queues 32"
for v in "a::--sweep 1,16384,8,-1,1" "b::--sweep 1,16384,8,-1,1 --link-pages 4k" "c::--sweep 1,16384,8,-1,1 --link-pages thp" "d::--sweep 2,16384,8,-1,2" "e::--sweep 2,16384,8,-1,2 --link-pages 4k" "f::--xproc 1 --sweep 1,16384,8,-1,1" "g::--xproc 1 --sweep 2,16384,8,-1,2" ; do
  tag=${v%%::*}; args=${v#*::}
  timeout -k 10 300 python -u tools/bench_tile.py $C $args --out $O/$tag.jsonl > $O/$tag.log 2>&1 || { echo RUN_FAILED $tag; tail -20 $O/$tag.log; exit 1; }
  python -c "
import json,sys
for l in open('$O/$tag.jsonl'):
  d=json.loads(l); print('$tag', d['tiles'], round(d['txns_per_s']/1e6,2), d['batch_latency_ms'], d.get('link_pages'), d.get('xproc'), d['published_ok'], d['counters'].get('rescued'))
"
done
