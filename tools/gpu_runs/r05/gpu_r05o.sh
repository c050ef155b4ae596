set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05o; mkdir -p $O
export TMPDIR=/tmp FDGPU_IO_DMA=0
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
P="python -u tools/io_probe.py --npz /tmp/cfg1.npz --out $O/io.jsonl"
for a in "--engines 1 --batches 400" "--engines 2 --batches 400"; do
  timeout -k 10 120 $P $a >> $O/io.log 2>&1 || { echo PROBE_FAILED $a; tail -20 $O/io.log; exit 1; }
done
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 -u tools/io_probe.py --npz /tmp/cfg1.npz --engines 2 --batches 200 --tag traced --out $O/io.jsonl > $O/trace.log 2>&1 || { echo TRACE_FAILED; tail -20 $O/trace.log; exit 1; }
cat $O/io.jsonl
find $O/trace -name "*stats.csv"
