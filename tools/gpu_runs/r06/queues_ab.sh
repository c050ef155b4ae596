#!/bin/bash
# The headline loop with 2, 3 and 4 device-resident copies on their own streams, alternating twice.
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do
  for q in 2 3 4; do
    timeout -k 10 300 python3 bench.py --no-extras --steps 30 --warmup 4 --queues $q > $out/q${q}_$r.json 2> $out/q${q}_$r.err \
      || { tail $out/q${q}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/q${q}_$r.json')); print('queues $q run $r', d['value'], d['ms_per_step'])"
  done
done
