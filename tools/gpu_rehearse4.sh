# Readiness check of the driver's multi-GPU bench path on ONE MI355X: 4 ranks
# via torch.distributed.run share the device round robin (bench.py), with
# reduced batch sizes so the whole line fits the box.  Not a scaling claim.
# usage: bash tools/gpu_rehearse8.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1; mkdir -p $o
echo "[$(date +%T)] 4 ranks on one GPU (each rank also starts a tile child process: 8 GPU processes)"
t0=$(date +%s)
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 4 --steps 5 --warmup 1 --txns 200000 --adv-txns 100000 \
  --keypool-txns 100000 --cfg3-txns 30000 --latency-batches 200 --cpu-sample 100000 \
  > $o/bench4.json 2> $o/bench4.err || { tail -30 $o/bench4.err; exit 1; }
t1=$(date +%s)
echo "wall_s $((t1 - t0))" | tee $o/bench4_wall.txt
cat $o/bench4.json
echo "[$(date +%T)] done"
