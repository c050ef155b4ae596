# round-3 call: bench with the tile lines in a child process
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03u; mkdir -p $o
echo "[$(date +%T)] bench"
timeout -k 10 900 python3 bench.py > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$o/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'])
for k,v in d.items():
    if k.startswith('tile_') and k != 'tile_config': print(' ', k, v)
for k,v in d.items():
    if 'latency' in k and not k.startswith('tile_'): print(' ', k, v)"
echo "[$(date +%T)] done"
