set -o pipefail
o=gpurun_out/g7; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "edges or cross" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 100000 --latency-batches 50 > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
cat $o/bench.json
