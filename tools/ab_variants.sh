#!/bin/bash
# GPU A/B of engine-library variants built by tools/build_variant.sh:
#   bash tools/ab_variants.sh main dsm2 fused ...   ("main" = the in-tree library)
# Per variant: bench.py --no-extras JSON + rocprofv3 kernel stats under gpurun_out/ab/<name>/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in "$@"; do
  lib=firedancer_amd/libfd_ed25519_gpu.so
  [ "$v" != main ] && lib=build/$v/libfd_ed25519_gpu.so
  d=gpurun_out/ab/$v; mkdir -p $d
  FDGPU_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d/prof -o run --output-format csv \
    -- python3 bench.py --no-extras --steps 10 --warmup 2 > $d/bench.json 2> $d/bench.err || { echo "FAIL $v"; exit 1; }
  echo "== $v: $(python3 -c "import json;d=json.load(open('$d/bench.json'));print(d['ms_per_step'],'ms/step',d['value'],d['self_check_codes'])")"
  f=$(find $d/prof -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'fdgpu' in r['Name']:
        print('   %-40s calls %5s avg %.3f ms' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e6))
PY
done
