# round-3 call: the bench's tile lines with the threads pinned to the box's least busy cores
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03ab; mkdir -p $o
for r in 1; do
  echo "[$(date +%T)] run $r"
  timeout -k 10 600 python3 bench.py --adv-txns 0 --keypool-txns 0 > $o/b$r.json 2> $o/b$r.err || { tail $o/b$r.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$o/b$r.json').read().strip().splitlines()[-1])
print(' value', d['value'], 'cpus', d['cpu_baseline'].get('cpus') if d.get('cpu_baseline') else None, 'mux1', d['tile_mux1_capacity_txns_per_s_runs'], 'mux2', d['tile_mux2_capacity_txns_per_s_runs'], 'ratio', d['tile_mux2_vs_mux1_capacity'], 'paced', d['tile_mux1_paced_16M_txns_per_s'], d['tile_mux2_paced_24M_txns_per_s'], 'lat', d['p99_batch_latency_ms'], d['p99_batch_latency_registered_ms'])"
done
echo "[$(date +%T)] done"
