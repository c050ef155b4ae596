#!/bin/bash
# Kernel A/B on one box: GPU parity of an A/B library, the headline loop
# alternating product / A/B, and one PMC pass set per build.
#   bash tools/gpu_runs/r06/ab_kernel.sh <tag> <ab-name> [tests]
# -> gpurun_out/<tag>/
set -o pipefail
tag=$1; ab=$2; what=${3:-}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
AB=build/ab/$ab/libfd_ed25519_gpu.so
step() { echo "[$(date +%T)] $*"; }
if [[ "$what" == *tests* ]]; then
  step tests product
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 \
    || { tail -40 $out/tests.log; exit 1; }
  tail -1 $out/tests.log
fi
step parity $ab
FDGPU_LIB=$PWD/$AB timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $out/parity_$ab.log 2>&1 || { tail -40 $out/parity_$ab.log; exit 1; }
tail -1 $out/parity_$ab.log
for r in 1 2; do
  step bench product $r
  timeout -k 10 300 python3 bench.py --no-extras --steps 20 --warmup 3 > $out/bench_prod_$r.json 2>$out/bench_prod_$r.err \
    || { tail $out/bench_prod_$r.err; exit 1; }
  step bench $ab $r
  FDGPU_LIB=$PWD/$AB timeout -k 10 300 python3 bench.py --ab-build --no-extras --steps 20 --warmup 3 \
    > $out/bench_${ab}_$r.json 2>$out/bench_${ab}_$r.err || { tail $out/bench_${ab}_$r.err; exit 1; }
  python3 -c "import json,sys;[print(f, json.load(open(f))['value'], json.load(open(f))['roofline']['frac']) for f in sys.argv[1:]]" \
    $out/bench_prod_$r.json $out/bench_${ab}_$r.json
done
P=(FETCH_SIZE WRITE_SIZE "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES")
for b in prod $ab; do
  lib=$PWD/firedancer_amd/libfd_ed25519_gpu.so; [ $b = prod ] || lib=$PWD/$AB
  dirs=()
  for i in "${!P[@]}"; do
    step pmc $b pass $i: ${P[$i]}
    FDGPU_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc ${P[$i]} -d $out/pmc_${b}_$i -o run --output-format csv \
      -- python3 bench.py --ab-build --no-extras --queues 1 --steps 3 --warmup 1 > $out/pmc_${b}_$i.json 2>$out/pmc_${b}_$i.err \
      || { tail $out/pmc_${b}_$i.err; exit 1; }
    dirs+=($out/pmc_${b}_$i)
  done
  PMC_OUT_DIR=$out python3 tools/pmc_summary.py ${tag}_$b "${dirs[@]}" > $out/pmc_${b}_summary.txt || exit 1
  cat $out/pmc_${b}_summary.txt | head -30
done
step done
