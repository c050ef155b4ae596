# Readiness check of the driver's `--gpus 8` line WITH the tile lines, on ONE
# MI355X: 8 ranks via torch.distributed.run share the
# device round robin (bench.py), reduced sizes.  A sampler counts this job's
# processes that hold the GPU (/dev/kfd mapped) twice a second: the box allows
# 16.  Not a scaling claim.
# usage: bash tools/gpu_rehearse8_tiles.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1; mkdir -p $o
python3 - > $o/gpu_procs.txt 2>&1 <<'PY' &
import os, time
peak, t0, last = 0, time.time(), 0
while time.time() - t0 < 1000:
    n = 0
    for p in os.listdir("/proc"):
        if not p.isdigit():
            continue
        try:
            with open(f"/proc/{p}/maps") as f:
                held = "/dev/kfd" in f.read()
            if not held:                   # an open driver fd counts too (the box's process guard counts those)
                for fd in os.listdir(f"/proc/{p}/fd"):
                    t = os.readlink(f"/proc/{p}/fd/{fd}")
                    if t == "/dev/kfd" or t.startswith("/dev/dri/"):
                        held = True
                        break
            n += held
        except OSError:
            pass
    peak = max(peak, n)
    if time.time() - last > 5:
        print(f"t={time.time() - t0:.0f}s gpu_procs={n} peak={peak}", flush=True)
        last = time.time()
    time.sleep(0.2)
PY
sampler=$!
echo "[$(date +%T)] 8 ranks on one GPU, tile lines on"
t0=$(date +%s)
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 8 --steps 5 --warmup 1 --txns 200000 --adv-txns 100000 \
  --keypool-txns 100000 --cfg3-txns 30000 --tile-cfg3-txns 30000 --latency-batches 200 --cpu-sample 100000 \
  --node-lines 1 --node-procs 4 \
  > $o/bench8.json 2> $o/bench8.err
rc=$?
t1=$(date +%s)
kill $sampler
echo "wall_s $((t1 - t0)) rc $rc" | tee $o/bench8_wall.txt
tail -1 $o/gpu_procs.txt
[ $rc -eq 0 ] || { tail -30 $o/bench8.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$o/bench8.json').read().strip().splitlines()[-1])
print({k: d[k] for k in ('value','n_gpus','ms_per_step','parity_checked_txns','parity_mismatches','tile_published_ok_all_ranks','tile_mux1_capacity_txns_per_s_node') if k in d})
print({k: v for k, v in d.items() if k.startswith('tile_node')})
"
