# A/B on one MI355X box: parity tests of one variant, then bench of each
# variant, then phase stamps of stamps builds.
# usage: bash tools/gpu_ab.sh <outdir> <test-variant|-> "<bench variants>" "<stamps variant:path ...>"
#   variant "main" = firedancer_amd/libfd_ed25519_gpu.so, else build/<v>/libfd_ed25519_gpu.so
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1; mkdir -p $o
lib_of() { [ "$1" = main ] && echo firedancer_amd/libfd_ed25519_gpu.so || echo build/$1/libfd_ed25519_gpu.so; }
if [ "$2" != "-" ]; then
  echo "[$(date +%T)] parity tests ($2)"
  FDGPU_LIB=$(lib_of $2) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread > $o/tests_$2.log 2>&1 || { tail -30 $o/tests_$2.log; exit 1; }
  tail -1 $o/tests_$2.log
fi
for v in $3; do
  echo "[$(date +%T)] bench $v"
  FDGPU_LIB=$(lib_of $v) timeout -k 10 200 python3 bench.py --no-extras --steps 20 --warmup 3 > $o/bench_$v.json 2> $o/bench_$v.err || { tail $o/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$o/bench_$v.json'));print('$v',d['ms_per_step'],d['value'],d['roofline']['note'][-110:])"
done
for vp in $4; do
  n=${vp%%:*}; p=${vp##*:}
  echo "[$(date +%T)] stamps $n"
  FDGPU_LIB=build/$n/libfd_ed25519_gpu.so timeout -k 10 200 python3 tools/phase_stamps.py --path $p --out $o/stamps_$n.json > /dev/null 2> $o/stamps_$n.err || { tail $o/stamps_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$o/stamps_$n.json'));print('$n', d['verify_ms'], d['wave_life_cycles_mean'], {k:v['share'] for k,v in d['phases'].items()})"
done
