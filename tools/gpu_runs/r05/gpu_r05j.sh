set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ingest.py tests/test_tile_gpu.py tests/test_engine_proc.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|assert|FAIL" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --depth-lg-paced 14 --paced-reps 4 --pair 2 --spread 2 --wait-us 200 --reps 3 --hw-queues 32 --producers-same-as-tiles 1"
S="1,16384,8,12e6,2;2,16384,8,24e6,4;1,16384,8,-1,1;2,16384,8,-1,2"
for v in "dma::X=1" "load::FDGPU_IO_DMA=0"; do
  tag=${v%%::*}; envs=${v#*::}
  timeout -k 10 300 env $envs python -u tools/bench_tile.py $C --sweep "$S" --out $O/$tag.jsonl > $O/$tag.log 2>&1 || { echo RUN_FAILED $tag; tail -5 $O/$tag.log; exit 1; }
  python -c "
import json
for l in open('$O/$tag.jsonl'):
  d=json.loads(l); c=d['counters']; print('$tag', d['tiles'], d['rate_target'], round(d['txns_per_s']/1e6,2), d['batch_latency_ms'], d['published_ok'], c['overrun'], c.get('lap_margin_min'), round(c['submit_ns']/c['batches']/1e3,1))
"
done
