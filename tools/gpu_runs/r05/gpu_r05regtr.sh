# Registered host-fed feed, traced (kernels + memory copies), after the big-batch streams
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05regtr; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/host_fed_probe.py --ring 3 --feed registered,staged --steps 12 > $O/probe.log 2>&1 || { echo PROBE_FAILED; tail $O/probe.log; exit 1; }
cat $O/probe.log | tail -4
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o run -- python3 -u tools/host_fed_probe.py --ring 3 --feed registered --steps 12 > $O/tr.log 2>&1 || { echo TRACE_FAILED; tail $O/tr.log; exit 1; }
tail -2 $O/tr.log
find $O/tr -name "*.csv" | head
