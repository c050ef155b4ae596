set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05c3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/make_tile_npz.py --multi 1 --txns 250000 --out /tmp/cfg3s.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --multi 1 --batch-sig-max 32768 --payload-npz /tmp/cfg3s.npz --depth-lg 21 --wait-us 200 --reps 5 --hw-queues 32 --producers-same-as-tiles 1 --pin 1 --pair 2 --spread 2"
for pr in 4 1; do
  timeout -k 10 200 python -u tools/bench_tile.py $C --prefill-reps $pr --sweep "1,16384,8,-1,1,32768;2,16384,8,-1,2,24576" --out $O/p$pr.jsonl > $O/p$pr.log 2>&1 || { echo RUN_FAILED $pr; tail -5 $O/p$pr.log; exit 1; }
  python -c "
import json
for l in open('$O/p$pr.jsonl'):
  d=json.loads(l); print('reps $pr', d['tiles'], d['txns'], round(d['sigs_per_s']/1e6,2), d['batch_latency_ms'], d['published_ok'], d['counters']['overrun'])
"
done
