set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/host_fed_probe.py --ring 2,3,4 --arena-pages 4k,thp --reps 2 > $O/hf_sweep.jsonl 2> $O/hf_sweep.err || { echo PROBE_FAILED; tail -20 $O/hf_sweep.err; exit 1; }
cat $O/hf_sweep.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof_hf -o hf -- python tools/host_fed_probe.py --ring 3 --feed registered --steps 8 > $O/prof_hf.log 2>&1 || { echo PROF_FAILED; tail -20 $O/prof_hf.log; exit 1; }
tail -3 $O/prof_hf.log
