# Tile capacity A/B, second box: identity-sharing library vs head (reverted), alternating, 3 reps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05tcap3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --pair 2 --spread 2 --wait-us 200 --reps 2 --hw-queues 32 --producers-same-as-tiles 1 --pin 1 --warm-runs 1"
for rep in 1 2 3; do for v in "head::firedancer_amd/libfd_ed25519_gpu.so" "ident::build/ident/libfd_ed25519_gpu.so"; do
  tag=${v%%::*}; lib=${v#*::}
  FDGPU_LIB=$lib timeout -k 10 170 python -u tools/bench_tile.py $C --sweep "1,16384,8,-1,1;2,16384,8,-1,2" --out $O/${tag}_$rep.jsonl > $O/${tag}_$rep.log 2>&1; rc=$?; [ $rc -le 1 ] || { echo RUN_FAILED $tag; tail -5 $O/${tag}_$rep.log; exit 1; }
  python -c "
import json
r=[json.loads(l) for l in open('$O/${tag}_$rep.jsonl')]
print('$tag', $rep, [(d['tiles'], round(d['txns_per_s']/1e6,1)) for d in r])
"
done; done
