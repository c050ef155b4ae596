set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r02c; mkdir -p $o
echo "[$(date +%T)] hs2 parity tests"
FDGPU_LIB=build/hs2/libfd_ed25519_gpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread > $o/tests_hs2.log 2>&1 || { tail -30 $o/tests_hs2.log; exit 1; }
tail -1 $o/tests_hs2.log
for v in main hs1 hs2; do
  lib=firedancer_amd/libfd_ed25519_gpu.so; [ $v != main ] && lib=build/$v/libfd_ed25519_gpu.so
  echo "[$(date +%T)] bench $v"
  FDGPU_LIB=$lib timeout -k 10 200 python3 bench.py --no-extras --steps 20 --warmup 3 > $o/bench_$v.json 2> $o/bench_$v.err || { tail $o/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$o/bench_$v.json'));print('$v',d['ms_per_step'],d['value'],d['roofline']['note'][-120:])"
done
for v in hs2stamps:hs rastamps:ra; do
  n=${v%%:*}; p=${v##*:}
  echo "[$(date +%T)] stamps $n"
  FDGPU_LIB=build/$n/libfd_ed25519_gpu.so timeout -k 10 200 python3 tools/phase_stamps.py --path $p --out $o/stamps_$n.json > /dev/null 2> $o/stamps_$n.err || { tail $o/stamps_$n.err; exit 1; }
  cat $o/stamps_$n.json
done
