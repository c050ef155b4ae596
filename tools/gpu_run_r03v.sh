# round-3 call: mux tile batch growth under load, A/B (FDT_VMUX_GROW=0: the plain batch timer)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03v; mkdir -p $o
for g in 0 1 0 1; do
  echo "[$(date +%T)] grow=$g"
  FDT_VMUX_GROW=$g timeout -k 10 300 python3 tools/bench_tile.py --mux 1 --gpu-parse 2 --multi 0 --txns 1000000 --depth-lg 21 --depth-lg-paced 19 --reps 2 \
    --producers-same-as-tiles 1 --sweep "1,16384,8,-1;2,16384,8,-1;1,16384,8,16e6,2;2,16384,8,32e6,4" --out $o/g$g.jsonl > $o/g$g.log 2>&1 || { tail $o/g$g.log; exit 1; }
  python3 -c "
import json
for l in open('$o/g$g.jsonl'):
    d=json.loads(l); c=d['counters']; b=max(1,c['batches'])
    print(' tiles', d['tiles'], 'P', d['producers'], 'rate', d['rate_target'], round(d['txns_per_s']/1e6,2), 'M', d['batch_latency_ms'], 'txn/batch', round(d['txns']/b), 'gpu ms %.3f' % (c['batch_gpu_ns']/b/1e6), 'ovr', c['overrun'], 'pub_ok', c['published']==d['expected_published'])"
done
echo "[$(date +%T)] done"
