export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04an; mkdir -p $O
python3 - <<'PY'
import sys, os, numpy as np
sys.path.insert(0,'.')
from firedancer_amd import workload
a,t,m=workload.cfg1(1000000, seed=0x5EED0005)
ps=workload.payloads(a,t); pa,po,psz=workload.pack_payloads(ps)
np.savez('/tmp/cfg1.npz', arena=pa, offs=po, sizes=psz, modes=m, n_sig=int(t["sig_cnt"].sum()))
cpus = workload.same_l3_first(sorted(os.sched_getaffinity(0)), 6)
open('/tmp/cpus.txt','w').write(",".join(str(c) for c in cpus))
print("cpus", cpus)
PY
CPUS=$(cat /tmp/cpus.txt)
B="python -u tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 0 --producers-same-as-tiles 1 --depth-lg 21 --depth-lg-paced 14 --paced-reps 4 --wait-us 200 --pin 1 --hw-queues 32 --reps 5 --pair 2 --spread 2 --payload-npz /tmp/cfg1.npz --txns 1000000 --cpu-list $CPUS"
SW="1,16384,8,12e6,2;1,16384,8,16e6,2;2,16384,8,20e6,4;2,16384,8,24e6,4"
for V in cur lto base cur lto base; do
  case $V in cur) L=$R/firedancer_amd/libfd_verify_tile.so;; lto) L=$R/tools/scratch/wt_lto/firedancer_amd/libfd_verify_tile.so;; base) L=$R/tools/scratch/wt_base/firedancer_amd/libfd_verify_tile.so;; esac
  FDGPU_TILE_LIB=$L timeout -k 10 200 $B --sweep "$SW" --out $O/$V.$RANDOM.jsonl > /dev/null 2>> $O/err.log || echo "rc=$? $V" >> $O/err.log
done
exit 0
