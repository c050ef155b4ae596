set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
timeout -k 10 300 env FDGPU_AUX_CUS=8 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_tile_gpu.py tests/test_gpu_ingest.py > $O/aux_tests.log 2>&1 || { echo AUX_TESTS_FAILED; tail -20 $O/aux_tests.log; exit 1; }
tail -1 $O/aux_tests.log
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --depth-lg-paced 14 --paced-reps 4 --pair 2 --spread 2 --wait-us 200 --reps 3 --hw-queues 32 --producers-same-as-tiles 1"
S="2,16384,8,24e6,4;1,16384,8,-1,1;2,16384,8,-1,2"
for v in "base::X=1" "aux8::FDGPU_AUX_CUS=8" "aux16::FDGPU_AUX_CUS=16" "aux4::FDGPU_AUX_CUS=4"; do
  tag=${v%%::*}; envs=${v#*::}
  timeout -k 10 300 env $envs python -u tools/bench_tile.py $C --sweep "$S" --out $O/$tag.jsonl > $O/$tag.log 2>&1 || { echo RUN_FAILED $tag; tail -20 $O/$tag.log; exit 1; }
  python -c "
import json
for l in open('$O/$tag.jsonl'):
  d=json.loads(l); c=d['counters']; print('$tag', d['tiles'], d['rate_target'], round(d['txns_per_s']/1e6,2), d['batch_latency_ms'], d['published_ok'], c['overrun'], c.get('lap_margin_min'))
"
done
