set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/host_fed_probe.py --ring 3 --feed registered,staged --arena-pages 4k,thp --steps 12 --reps 2 > $O/hf.log 2>&1 || { echo HF_FAILED; tail -20 $O/hf.log; exit 1; }
cat $O/hf.log | grep -v "^\[" | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run --output-format csv -- python3 -u tools/host_fed_probe.py --ring 3 --feed registered,staged --arena-pages 4k --steps 8 > $O/hf_trace.log 2>&1 || { echo TRACE_FAILED; tail -20 $O/hf_trace.log; exit 1; }
ls $O/trace/*/ 2>/dev/null | head; find $O/trace -name "*.csv" | head
