set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05hf5; mkdir -p $O
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8
for rep in 1 2; do for v in "c16::FDGPU_COPY_CHUNK_MB=16" "c0::FDGPU_COPY_CHUNK_MB=0" "c8::FDGPU_COPY_CHUNK_MB=8" "c32::FDGPU_COPY_CHUNK_MB=32"; do
  tag=${v%%::*}; envs=${v#*::}
  timeout -k 10 300 env $envs python -u tools/host_fed_probe.py --ring 3 --feed staged --steps 16 --reps 2 > $O/hf_${tag}_$rep.log 2>&1 || { echo HF_FAILED; tail -20 $O/hf_${tag}_$rep.log; exit 1; }
  grep '^{' $O/hf_${tag}_$rep.log | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); print('$tag', d['feed'], d['ring'], round(d['sigs_per_s']/1e6,1), d['ms_per_batch'], d['codes_equal'])
"
done; done
timeout -k 10 120 python3 bench.py --no-extras --steps 20 --warmup 3 > $O/dev.json 2>$O/dev.err && tail -1 $O/dev.json | cut -c1-120
