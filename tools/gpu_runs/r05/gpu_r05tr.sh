set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05tr; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --pair 2 --spread 2 --wait-us 200 --reps 2 --hw-queues 32 --producers-same-as-tiles 1 --pin 1 --warm-runs 1"
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tile -o run --output-format csv -- python3 -u tools/bench_tile.py $C --sweep "2,16384,8,-1,2" --out $O/tile.jsonl > $O/tile.log 2>&1 || { echo TRACE_FAILED; tail -20 $O/tile.log; exit 1; }
GPU_MAX_HW_QUEUES=32 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/probe -o run --output-format csv -- python3 -u tools/io_probe.py --npz /tmp/cfg1.npz --engines 2 --batches 200 --out $O/probe.jsonl > $O/probe.log 2>&1 || { echo TRACE2_FAILED; tail -20 $O/probe.log; exit 1; }
grep -o '"txns_per_s": [0-9.]*' $O/tile.jsonl $O/probe.jsonl
