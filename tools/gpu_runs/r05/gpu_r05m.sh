set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05m; mkdir -p $O
export TMPDIR=/tmp FDGPU_IO_DMA=0
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --pair 2 --spread 2 --wait-us 200 --reps 1 --hw-queues 32 --producers-same-as-tiles 1"
timeout -s KILL 170 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc -o run --output-format csv -- python3 -u tools/bench_tile.py $C --sweep "2,16384,8,-1,2" --out $O/pmc.jsonl > $O/pmc.log 2>&1 || { echo PMC_FAILED; tail -20 $O/pmc.log; exit 1; }
find $O/pmc -name "*.csv" | head
