set -o pipefail
o=gpurun_out/g8; mkdir -p $o
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
for n in 917504 1000000 1048576 2000000; do
  timeout -k 10 200 python bench.py --no-extras --steps 10 --warmup 2 --txns $n > $o/b_$n.json 2>$o/b_$n.err || { tail $o/b_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$o/b_$n.json'));print($n, d['ms_per_step'], round(d['ms_per_step']*1e6/$n,4), 'ms per 1M')"
done
