set -o pipefail
o=gpurun_out/g2; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_tile_gpu.py -x -v --timeout 120 --timeout-method thread > $o/tile_tests.log 2>&1 || { tail -30 $o/tile_tests.log; exit 1; }
tail -2 $o/tile_tests.log
timeout -k 10 200 python -u tools/bench_tile.py --gpus 1 --tiles 1 --txns 200000 --out $o/tile_cfg3_t1.json > $o/bt1.log 2>&1; tail -1 $o/bt1.log
timeout -k 10 200 python -u tools/bench_tile.py --gpus 1 --tiles 2 --txns 200000 --out $o/tile_cfg3_t2.json > $o/bt2.log 2>&1; tail -1 $o/bt2.log
timeout -k 10 200 python -u tools/bench_tile.py --gpus 1 --tiles 1 --multi 0 --txns 1000000 --out $o/tile_cfg1_t1.json > $o/bt3.log 2>&1; tail -1 $o/bt3.log
timeout -k 10 200 python -u tools/bench_tile.py --gpus 1 --tiles 4 --multi 0 --txns 1000000 --out $o/tile_cfg1_t4.json > $o/bt4.log 2>&1; tail -1 $o/bt4.log
