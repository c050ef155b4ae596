#!/bin/bash
# Engine-policy bring-up (report mode, incl. teardown) and the large-message sync test.
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
echo "[$(date +%T)] sandbox report"
timeout -k 10 300 python -u tools/sandbox_report.py --modes 2 > $out/sandbox.jsonl 2> $out/sandbox.err || { tail -30 $out/sandbox.err; cat $out/sandbox.jsonl; exit 1; }
cat $out/sandbox.jsonl
echo "[$(date +%T)] sync large"
timeout -k 10 400 python -u -m pytest tests/test_gpu_sync_large.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/sync_large.log 2>&1 || { tail -40 $out/sync_large.log; exit 1; }
tail -2 $out/sync_large.log
echo "[$(date +%T)] done"
