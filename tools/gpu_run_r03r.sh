# round-3 call: tile-less pipeline capacity vs hardware queues, and a 16-queue trace
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03r; mkdir -p $o
echo "[$(date +%T)] gather-path GPU tests"
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_ingest.py tests/test_tile_gpu.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for q in 16 32; do
  echo "[$(date +%T)] pipeline capacity, $q hw queues"
  timeout -k 10 300 python3 tools/pipe_conc.py --batches 240 --hw-queues $q \
    --runs "1,8,16384;1,16,16384;2,8,16384;1,8,32768;2,8,32768;1,4,65536;2,4,65536" --out $o/pipe.jsonl > $o/pipe$q.log 2>&1 || { tail $o/pipe$q.log; exit 1; }
  cat $o/pipe$q.log
done
echo "[$(date +%T)] trace 1,16,16384 at 16 queues"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/t16 -o run -- \
  python3 tools/pipe_conc.py --batches 160 --hw-queues 16 --runs "1,16,16384" > $o/t16.log 2>&1 || { tail $o/t16.log; exit 1; }
grep -v "^[EWI]2026" $o/t16.log | tail -2
echo "[$(date +%T)] done"
