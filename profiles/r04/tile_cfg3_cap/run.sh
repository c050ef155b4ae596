export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04aq; mkdir -p $O
python3 - <<'PY'
import sys, numpy as np
sys.path.insert(0,'.')
from firedancer_amd import workload
a,t,m=workload.cfg3(150000, seed=workload.CFG3_SEED)
ps=workload.payloads(a,t); pa,po,psz=workload.pack_payloads(ps)
np.savez('/tmp/cfg3.npz', arena=pa, offs=po, sizes=psz, modes=m, n_sig=int(t["sig_cnt"].sum()))
PY
B="python -u tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 1 --producers-same-as-tiles 1 --depth-lg 21 --depth-lg-paced 14 --paced-reps 4 --wait-us 200 --pin 1 --hw-queues 32 --reps 5 --pair 2 --spread 2 --payload-npz /tmp/cfg3.npz --txns 150000"
for C in 24576 16384 12288 24576 16384 12288; do
  timeout -k 10 200 $B --batch-sig-max $C --sweep "1,16384,8,-1,1;2,16384,8,-1,2" --out $O/c$C.$RANDOM.jsonl > /dev/null 2>> $O/err.log || echo "rc=$? $C" >> $O/err.log
done
exit 0
