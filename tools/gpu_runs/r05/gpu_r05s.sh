set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05s; mkdir -p $O
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=32
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
P="python -u tools/io_probe.py --npz /tmp/cfg1.npz --out $O/io.jsonl --batches 300 --engines 2 --pair 0 --spread 0"
for v in "d16::FDGPU_AUX_BLOCKS_IN=16 FDGPU_AUX_BLOCKS_FIN=16" "d8::FDGPU_AUX_BLOCKS_IN=8 FDGPU_AUX_BLOCKS_FIN=8" "di8f16::FDGPU_AUX_BLOCKS_IN=8 FDGPU_AUX_BLOCKS_FIN=16" "di4f16::FDGPU_AUX_BLOCKS_IN=4 FDGPU_AUX_BLOCKS_FIN=16" "di8f12::FDGPU_AUX_BLOCKS_IN=8 FDGPU_AUX_BLOCKS_FIN=12" "di16f24::FDGPU_AUX_BLOCKS_IN=16 FDGPU_AUX_BLOCKS_FIN=24"; do
  tag=${v%%::*}; envs=${v#*::}
  timeout -k 10 120 env $envs $P --tag $tag >> $O/io.log 2>&1 || { echo PROBE_FAILED $tag; tail -20 $O/io.log; exit 1; }
done
timeout -k 10 120 env FDGPU_AUX_BLOCKS_IN=16 FDGPU_AUX_BLOCKS_FIN=16 $P --pair 2 --spread 2 --tag d16ps >> $O/io.log 2>&1 || { echo PROBE_FAILED ps; tail -20 $O/io.log; exit 1; }
timeout -k 10 120 env FDGPU_AUX_BLOCKS_IN=16 FDGPU_AUX_BLOCKS_FIN=16 $P --engines 1 --tag d16e1 >> $O/io.log 2>&1 || { echo PROBE_FAILED e1; tail -20 $O/io.log; exit 1; }
python -c "
import json
for l in open('$O/io.jsonl'):
  d=json.loads(l); print(d['tag'], round(d['txns_per_s']/1e6,1), d['batch_latency_ms'])
"
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --depth-lg-paced 14 --paced-reps 4 --pair 2 --spread 2 --wait-us 200 --reps 3 --hw-queues 32 --producers-same-as-tiles 1"
S="1,16384,8,12e6,2;2,16384,8,24e6,4;1,16384,8,-1,1;2,16384,8,-1,2"
for v in "tload::FDGPU_IO_DMA=0" "td16::FDGPU_AUX_BLOCKS_IN=16 FDGPU_AUX_BLOCKS_FIN=16" "tl16::FDGPU_IO_DMA=0 FDGPU_AUX_BLOCKS_IN=16 FDGPU_AUX_BLOCKS_FIN=16"; do
  tag=${v%%::*}; envs=${v#*::}
  timeout -k 10 170 env $envs python -u tools/bench_tile.py $C --sweep "$S" --out $O/$tag.jsonl > $O/$tag.log 2>&1 || { echo RUN_FAILED $tag; tail -5 $O/$tag.log; exit 1; }
  python -c "
import json
for l in open('$O/$tag.jsonl'):
  d=json.loads(l); c=d['counters']; print('$tag', d['tiles'], d['rate_target'], round(d['txns_per_s']/1e6,2), d['batch_latency_ms'], d['published_ok'])
"
done
