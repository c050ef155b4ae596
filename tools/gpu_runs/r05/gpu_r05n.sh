set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05n; mkdir -p $O
export TMPDIR=/tmp FDGPU_IO_DMA=0
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
P="python -u tools/io_probe.py --npz /tmp/cfg1.npz --out $O/io.jsonl --batches 96"
for a in "--engines 1" "--engines 2" "--engines 4" "--engines 1 --inflight 16" "--engines 2 --pair 0 --spread 0" "--engines 2 --batch 32768" "--engines 4 --pair 0 --spread 0"; do
  timeout -k 10 120 $P $a >> $O/io.log 2>&1 || { echo PROBE_FAILED $a; tail -20 $O/io.log; exit 1; }
done
timeout -k 10 120 env FDGPU_IO_DMA=1 $P --engines 2 --tag dma >> $O/io.log 2>&1 || { echo PROBE_FAILED dma; tail -20 $O/io.log; exit 1; }
cat $O/io.jsonl
