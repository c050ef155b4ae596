set -o pipefail
o=gpurun_out/g3; mkdir -p $o
timeout -k 10 400 python -u tools/bench_tile.py --gpus 1 --txns 1000000 --depth-lg 20 --out $o/tile_cfg3_sweep.jsonl \
  --sweep "1,4096,3,0;1,16384,3,0;1,32768,4,0;2,16384,3,0;1,4096,3,1000000;1,4096,3,2000000" > $o/sweep.log 2>&1; rc=$?; cat $o/sweep.log; exit $rc
