set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05r; mkdir -p $O
export TMPDIR=/tmp FDGPU_IO_DMA=0 GPU_MAX_HW_QUEUES=32
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
P="python -u tools/io_probe.py --npz /tmp/cfg1.npz --out $O/io.jsonl --batches 300 --engines 2 --pair 0 --spread 0"
for rep in 1 2; do
for v in "a64::X=1" "a32::FDGPU_AUX_BLOCKS_IN=32 FDGPU_AUX_BLOCKS_FIN=32" "a16::FDGPU_AUX_BLOCKS_IN=16 FDGPU_AUX_BLOCKS_FIN=16" "a8::FDGPU_AUX_BLOCKS_IN=8 FDGPU_AUX_BLOCKS_FIN=8" "i16f64::FDGPU_AUX_BLOCKS_IN=16" "i64f16::FDGPU_AUX_BLOCKS_FIN=16" "dma16::FDGPU_IO_DMA=1 FDGPU_AUX_BLOCKS_IN=16 FDGPU_AUX_BLOCKS_FIN=16"; do
  tag=${v%%::*}; envs=${v#*::}
  timeout -k 10 120 env $envs $P --tag $tag >> $O/io.log 2>&1 || { echo PROBE_FAILED $tag; tail -20 $O/io.log; exit 1; }
done; done
python -c "
import json
for l in open('$O/io.jsonl'):
  d=json.loads(l); print(d['tag'], round(d['txns_per_s']/1e6,1), d['batch_latency_ms'])
"
