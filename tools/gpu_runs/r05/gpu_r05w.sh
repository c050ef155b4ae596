set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05w; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --depth-lg-paced 14 --paced-reps 4 --pair 2 --spread 2 --wait-us 200 --reps 5 --hw-queues 32 --producers-same-as-tiles 1 --pin 1"
timeout -k 10 300 python -u tools/bench_tile.py $C --xproc 1 --sweep "2,16384,8,24e6,4;1,16384,8,16e6,2" --out $O/xp.jsonl > $O/xp.log 2>&1 || { echo RUN_FAILED xp; tail -5 $O/xp.log; exit 1; }
timeout -k 10 200 python -u tools/bench_tile.py $C --sweep "2,16384,8,24e6,4;1,16384,8,16e6,2" --out $O/ip.jsonl > $O/ip.log 2>&1 || { echo RUN_FAILED ip; tail -5 $O/ip.log; exit 1; }
python -c "
import json
for t in ('xp','ip'):
  for l in open('$O/'+t+'.jsonl'):
    d=json.loads(l); c=d['counters']; print(t, d['tiles'], d['rate_target'], round(d['txns_per_s']/1e6,2), d['batch_latency_ms'], 'margin', c.get('lap_margin_min'), 'rescued', c.get('rescued'), 'stall', c.get('stall_max_ns'), 'batches', c['batches'], 'overrun', c['overrun'])
"
