# Tile capacity vs pinning on a shared box: CPU busy fractions of our CPU share, then one tile
# pinned / unpinned alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05pin; mkdir -p $O
export TMPDIR=/tmp
python3 tools/cpu_busy.py > $O/busy0.json; cat $O/busy0.json
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --pair 2 --spread 2 --wait-us 200 --reps 2 --hw-queues 32 --producers-same-as-tiles 1 --warm-runs 1"
for rep in 1 2 3; do for pin in 1 0; do
  python3 tools/cpu_busy.py --secs 0.3 > $O/busy_${pin}_$rep.json
  timeout -k 10 170 python -u tools/bench_tile.py $C --pin $pin --sweep "1,16384,8,-1,1;2,16384,8,-1,2" --out $O/pin${pin}_$rep.jsonl > $O/pin${pin}_$rep.log 2>&1; rc=$?; [ $rc -le 1 ] || { echo RUN_FAILED; tail -5 $O/pin${pin}_$rep.log; exit 1; }
  python -c "
import json
r=[json.loads(l) for l in open('$O/pin${pin}_$rep.jsonl')]
b=json.load(open('$O/busy_${pin}_$rep.json'))
print('pin', $pin, $rep, [(d['tiles'], round(d['txns_per_s']/1e6,1)) for d in r], 'load', [round(x,1) for x in b['loadavg']], 'busy>0.5:', [c for c,v in b['busy'].items() if v>0.5])
"
done; done
