#!/bin/bash
# One GPU measurement round (run on the GPU box via gpurun):
#   bash tools/measure.sh <tag> [steps...]      steps: tests bench trace pmc (default: all)
# -> gpurun_out/<tag>/: tests.log, bench.json, trace2q/ + trace2q_summary.json (the
#    default two-queue timed loop), trace1q/ + kernel_stats.csv (one queue, isolated
#    launches), pmc passes + <tag>_pmc.json.
# Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
tag=$1; shift
what=${*:-tests bench trace pmc}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
has() { [[ " $what " == *" $1 "* ]]; }
if has tests; then
  step tests
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread > $out/tests.log 2>&1 \
    || { tail -40 $out/tests.log; exit 1; }
  tail -1 $out/tests.log
fi
if has bench; then
  step bench
  timeout -k 10 600 python3 bench.py > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; cat $out/bench.json; exit 1; }
  cat $out/bench.json
fi
if has trace; then
  step trace-2q
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace2q -o run --output-format csv \
    -- python3 bench.py --no-extras --steps 20 --warmup 3 > $out/trace2q_bench.json 2>$out/trace2q.err \
    || { tail $out/trace2q.err; exit 1; }
  python3 tools/trace_summary.py $out/trace2q $out/trace2q_bench.json $out/trace2q_summary.json || exit 1
  step trace-1q
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace1q -o run --output-format csv \
    -- python3 bench.py --no-extras --queues 1 --steps 10 --warmup 2 > $out/trace1q_bench.json 2>$out/trace1q.err \
    || { tail $out/trace1q.err; exit 1; }
  cp $(find $out/trace1q -name '*kernel_stats.csv' | head -1) $out/kernel_stats.csv
  python3 tools/trace_summary.py $out/trace1q $out/trace1q_bench.json $out/trace1q_summary.json > /dev/null || exit 1
fi
if has pmc; then
  P=(FETCH_SIZE WRITE_SIZE
     "SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT"
     "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR")
  dirs=()
  for i in "${!P[@]}"; do
    step pmc pass $i: ${P[$i]}
    timeout -s KILL 120 rocprofv3 --pmc ${P[$i]} -d $out/pmc_$i -o run --output-format csv \
      -- python3 bench.py --no-extras --queues 1 --steps 3 --warmup 1 > $out/pmc_$i.json 2>$out/pmc_$i.err \
      || { tail $out/pmc_$i.err; exit 1; }
    dirs+=($out/pmc_$i)
  done
  PMC_OUT_DIR=$out python3 tools/pmc_summary.py $tag "${dirs[@]}" > /dev/null || exit 1
fi
step done
