set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05z2; mkdir -p $O
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8
for rep in 1 2; do
for v in "big::X=1" "off::FDGPU_BIG_STREAMS=0"; do
  tag=${v%%::*}; envs=${v#*::}
  timeout -k 10 300 env $envs python -u tools/host_fed_probe.py --ring 3 --feed registered,staged --steps 12 --reps 2 > $O/hf_${tag}_$rep.log 2>&1 || { echo HF_FAILED $tag; tail -20 $O/hf_$tag.log; exit 1; }
  grep '^{' $O/hf_${tag}_$rep.log | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); print('$tag', d['feed'], d['ring'], round(d['sigs_per_s']/1e6,1), d['ms_per_batch'], d['codes_equal'])
"
done; done
