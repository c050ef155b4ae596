#!/bin/bash
# GPU tests incl. the engine-process pipeline, the one-queue kernel trace that
# bench's isolated launch timing is compared with, and a queue-count sweep.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/g12; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv \
  -- python3 bench.py --no-extras --queues 1 --steps 10 --warmup 2 > $out/trace_bench.json 2>$out/trace.err || { tail $out/trace.err; exit 1; }
cp $(find $out/trace -name '*kernel_stats.csv' | head -1) $out/kernel_stats.csv
for qn in 1 2 3 4; do
  timeout -k 10 200 python3 bench.py --no-extras --queues $qn --steps 30 --warmup 4 > $out/bench_q$qn.json 2>$out/bench_q$qn.err || { tail $out/bench_q$qn.err; exit 1; }
  echo "q$qn $(python3 -c "import json;d=json.load(open('$out/bench_q$qn.json'));print(d['value'],d['ms_per_step'],d['roofline']['note'][-120:])")"
done
