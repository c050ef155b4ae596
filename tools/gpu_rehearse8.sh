# Readiness check of the driver's 8-GPU bench path on ONE MI355X: 8 ranks
# via torch.distributed.run share the device round robin (bench.py), with
# reduced batch sizes so the whole line fits the box.  Not a scaling claim.
# usage: bash tools/gpu_rehearse8.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1; mkdir -p $o
echo "[$(date +%T)] 8 ranks on one GPU"
t0=$(date +%s)
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 8 --steps 5 --warmup 1 --txns 200000 --adv-txns 100000 \
  --keypool-txns 100000 --cfg3-txns 30000 --latency-batches 200 --cpu-sample 100000 \
  > $o/bench8.json 2> $o/bench8.err || { tail -30 $o/bench8.err; exit 1; }
t1=$(date +%s)
echo "wall_s $((t1 - t0))" | tee $o/bench8_wall.txt
cat $o/bench8.json
echo "[$(date +%T)] done"
