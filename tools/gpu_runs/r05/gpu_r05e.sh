set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --pair 2 --spread 2 --wait-us 200 --hw-queues 32"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python -u tools/bench_tile.py $C --reps 1 --sweep "2,16384,8,-1,2;1,16384,8,-1,1" --out $O/trace_runs.jsonl > $O/trace.log 2>&1 || { echo TRACE_FAILED; tail -20 $O/trace.log; exit 1; }
python3 tools/trace_conc.py $(ls $O/trace/*kernel_trace.csv | head -1) > $O/trace_summary.txt 2>&1; cat $O/trace_summary.txt | head -40
for v in "f::--xproc 1 --sweep 1,16384,8,-1,1" "g::--xproc 1 --sweep 2,16384,8,-1,2" "d::--sweep 2,16384,8,-1,2"; do
  tag=${v%%::*}; args=${v#*::}
  timeout -k 10 300 python -u tools/bench_tile.py $C --reps 3 $args --out $O/$tag.jsonl > $O/$tag.log 2>&1 || { echo RUN_FAILED $tag; tail -20 $O/$tag.log; exit 1; }
  python -c "
import json,sys
for l in open('$O/$tag.jsonl'):
  d=json.loads(l); print('$tag', d['tiles'], round(d['txns_per_s']/1e6,2), d['batch_latency_ms'], d.get('xproc'), d['published_ok'], d['wall_s'])
"
done
