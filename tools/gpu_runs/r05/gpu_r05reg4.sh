# Registered / staged host-fed feed vs the process's HIP hardware queues (probe has one engine)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05reg4; mkdir -p $O
export TMPDIR=/tmp
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 -u tools/host_fed_probe.py --ring 3 --feed registered,staged --steps 12 --reps 2 > $O/probe_q$q.log 2>&1 || { echo PROBE_FAILED; tail $O/probe_q$q.log; exit 1; }
  echo "queues $q"; grep feed $O/probe_q$q.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  ', d['feed'], d['rep'], round(d['sigs_per_s'] / 1e6, 1), d['ms_per_batch'])"
done
