#!/bin/bash
# Engine sandbox bring-up (report, then enforce) and the full bench line.
#   bash tools/gpu_runs/r06/sandbox_bench.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
echo "[$(date +%T)] sandbox report"
timeout -k 10 300 python -u tools/sandbox_report.py > $out/sandbox.jsonl 2> $out/sandbox.err || { tail -30 $out/sandbox.err; cat $out/sandbox.jsonl; exit 1; }
cat $out/sandbox.jsonl
bash tools/gpu_runs/r06/bench_full.sh $tag
