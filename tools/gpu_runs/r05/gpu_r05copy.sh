# Host-fed staging threads 4 (head) vs 8, alternating, probe at bench.py's 8 HIP queues
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05copy; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do for v in "t4::firedancer_amd/libfd_ed25519_gpu.so" "t8::build/copy8/libfd_ed25519_gpu.so"; do
  tag=${v%%::*}; lib=${v#*::}
  FDGPU_LIB=$lib GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 -u tools/host_fed_probe.py --ring 3 --feed staged,registered --steps 12 --reps 2 > $O/${tag}_$i.log 2>&1 || { echo PROBE_FAILED; tail $O/${tag}_$i.log; exit 1; }
  grep feed $O/${tag}_$i.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('$tag', $i, d['feed'], d['rep'], round(d['sigs_per_s'] / 1e6, 1), d['submit_stage_expand_enqueue_ms'])"
done; done
