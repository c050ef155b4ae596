set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05q; mkdir -p $O
export TMPDIR=/tmp FDGPU_IO_DMA=0 GPU_MAX_HW_QUEUES=32
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
timeout -k 10 150 rocprofv3 --kernel-trace -d $O/t1 -o run --output-format csv -- python3 -u tools/io_probe.py --npz /tmp/cfg1.npz --engines 2 --pair 0 --spread 0 --batches 300 --tag traced --out $O/io.jsonl > $O/trace.log 2>&1 || { echo TRACE_FAILED; tail -20 $O/trace.log; exit 1; }
timeout -k 10 150 rocprofv3 --kernel-trace -d $O/t2 -o run --output-format csv -- python3 -u tools/io_probe.py --npz /tmp/cfg1.npz --engines 1 --inflight 16 --pair 0 --spread 0 --batches 300 --tag traced16 --out $O/io.jsonl > $O/trace2.log 2>&1 || { echo TRACE_FAILED; tail -20 $O/trace2.log; exit 1; }
cat $O/io.jsonl
