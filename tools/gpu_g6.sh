set -o pipefail
o=gpurun_out/g6; mkdir -p $o
FDGPU_LIB=build/kwin5/libfd_ed25519_gpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $o/tests_kwin5.log 2>&1 || { tail -30 $o/tests_kwin5.log; exit 1; }
tail -1 $o/tests_kwin5.log
bash tools/ab_variants.sh main kwin5 main kwin5
