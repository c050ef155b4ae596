set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05hf2; mkdir -p $O
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run --output-format csv -- python3 -u tools/host_fed_probe.py --ring 3 --feed staged,registered --arena-pages 4k --steps 10 > $O/hf_trace.log 2>&1 || { echo TRACE_FAILED; tail -20 $O/hf_trace.log; exit 1; }
grep '^{' $O/hf_trace.log | cut -c1-200
