#!/bin/bash
# One GPU measurement round (run on the GPU box via gpurun):
#   bash tools/measure.sh <tag>        e.g. r01
# -> gpurun_out/<tag>/: tests.log, kernel_stats.csv, pmc passes + <tag>_pmc.json, bench.json
# Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
tag=$1
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step tests
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
step kernel-trace
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv \
  -- python3 bench.py --no-extras --queues 1 --steps 10 --warmup 2 > $out/trace_bench.json 2>$out/trace.err || { tail $out/trace.err; exit 1; }
cp $(find $out/trace -name '*kernel_stats.csv' | head -1) $out/kernel_stats.csv
P=(FETCH_SIZE WRITE_SIZE
   "SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT"
   "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR")
dirs=()
for i in "${!P[@]}"; do
  step pmc pass $i: ${P[$i]}
  timeout -s KILL 120 rocprofv3 --pmc ${P[$i]} -d $out/pmc_$i -o run --output-format csv \
    -- python3 bench.py --no-extras --queues 1 --steps 3 --warmup 1 > $out/pmc_$i.json 2>$out/pmc_$i.err || { tail $out/pmc_$i.err; exit 1; }
  dirs+=($out/pmc_$i)
done
PMC_OUT_DIR=profiles python3 tools/pmc_summary.py $tag "${dirs[@]}" > /dev/null && cp profiles/${tag}_pmc.json $out/
step bench
timeout -k 10 400 python3 bench.py > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
cat $out/bench.json
