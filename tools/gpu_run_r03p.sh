# round-3 call: the gathered-frag GPU pipeline's capacity without a tile (tools/pipe_conc.py)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03p; mkdir -p $o
echo "[$(date +%T)] pipeline capacity"
timeout -k 10 400 python3 tools/pipe_conc.py --batches 240 \
  --runs "1,4,16384;1,8,16384;1,16,16384;2,4,16384;2,8,16384;4,4,16384;1,4,32768;1,4,65536;2,8,8192;1,2,65536" \
  --out $o/pipe.jsonl > $o/pipe.log 2>&1 || { tail $o/pipe.log; exit 1; }
cat $o/pipe.log
echo "[$(date +%T)] done"
