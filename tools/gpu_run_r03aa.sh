# round-3 call: the bench's tile lines vs the hardware queues the parent process holds (4 vs 8)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03aa; mkdir -p $o
for q in 4 8 4 8; do
  echo "[$(date +%T)] parent hw queues $q"
  timeout -k 10 600 python3 bench.py --hw-queues $q --adv-txns 0 --keypool-txns 0 > $o/b$q.json 2> $o/b$q.err || { tail $o/b$q.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$o/b$q.json').read().strip().splitlines()[-1])
print(' value', d['value'], 'mux1', d['tile_mux1_capacity_txns_per_s_runs'], 'mux2', d['tile_mux2_capacity_txns_per_s_runs'], 'ratio', d['tile_mux2_vs_mux1_capacity'], 'paced', d['tile_mux1_paced_16M_txns_per_s'], d['tile_mux2_paced_24M_txns_per_s'], d['tile_mux2_paced_24M_overruns'], 'pcie', d.get('pcie_inclusive_sigs_per_s_per_gpu'), d.get('pcie_inclusive_registered_sigs_per_s_per_gpu'))"
done
echo "[$(date +%T)] done"
