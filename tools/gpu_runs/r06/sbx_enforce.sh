#!/bin/bash
# Engine policy: report then enforce mode; the whole -m gpu suite (policy on by default); smoke + full bench.
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
echo "[$(date +%T)] sandbox report + enforce"
timeout -k 10 300 python -u tools/sandbox_report.py --modes 2,1 > $out/sandbox.jsonl 2> $out/sandbox.err || { tail -30 $out/sandbox.err; cat $out/sandbox.jsonl; exit 1; }
cut -c1-400 $out/sandbox.jsonl
echo "[$(date +%T)] gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
bash tools/gpu_runs/r06/bench_full.sh $tag
