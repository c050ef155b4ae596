# round-3 call: kernel traces of the tile-less gathered-frag pipeline, 16 K and 64 K batches
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03q; mkdir -p $o
for r in "1,8,16384" "1,4,65536"; do
  n=$(echo $r | tr , _)
  echo "[$(date +%T)] trace $r"
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $o/t$n -o run -- \
    python3 tools/pipe_conc.py --batches 120 --runs "$r" > $o/t$n.log 2>&1 || { tail $o/t$n.log; exit 1; }
  tail -1 $o/t$n.log
done
echo "[$(date +%T)] done"
