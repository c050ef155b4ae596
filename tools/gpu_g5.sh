set -o pipefail
o=gpurun_out/g5; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
bash tools/ab_variants.sh main noravoid
