set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05hf3; mkdir -p $O
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8
for rep in 1 2; do
  timeout -k 10 300 python -u tools/host_fed_probe.py --ring 3,4,5 --feed staged,registered --steps 16 --reps 1 > $O/hf_$rep.log 2>&1 || { echo HF_FAILED; tail -20 $O/hf_$rep.log; exit 1; }
  grep '^{' $O/hf_$rep.log | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); print(d['feed'], d['ring'], round(d['sigs_per_s']/1e6,1), d['ms_per_batch'], d['codes_equal'])
"
done
