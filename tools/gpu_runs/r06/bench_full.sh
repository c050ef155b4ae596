#!/bin/bash
# The driver's round-end sequence on one box: smoke, then the default bench line.
#   bash tools/gpu_runs/r06/bench_full.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -30 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
echo "[$(date +%T)] bench"
timeout -k 10 900 python3 bench.py > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; cat $out/bench.json; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_mismatches'))
for k, v in sorted(d.items()):
    if k.startswith('tile_xproc'): print(k, v)"
echo "[$(date +%T)] done"
