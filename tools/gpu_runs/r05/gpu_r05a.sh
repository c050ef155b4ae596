set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05a; mkdir -p $O
python -c "from firedancer_amd import tile; import json; print(json.dumps(tile.hugepage_support()))" > $O/huge.json 2>&1
df -h /dev/shm >> $O/huge.json 2>&1; nproc >> $O/huge.json
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_engine_proc.py tests/test_gpu_ingest.py tests/test_tile_gpu.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail -30 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline']['frac'])
for k,v in d.items():
  if k.startswith('host_fed') or 'xproc' in k or k.startswith('tile_mux'):
    print(k, v)
"
