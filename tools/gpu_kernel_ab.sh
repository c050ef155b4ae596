# Kernel A/B on one box: parity tests of each variant (the parity suite's
# golden / cross-product / fallback cases), then bench --no-extras of every
# variant twice, interleaved, and one PMC pass (VALU instructions) each.
# usage: bash tools/gpu_kernel_ab.sh <outdir> "<variants>"   (main = in-tree library)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/$1; mkdir -p $o
lib_of() { [ "$1" = main ] && echo firedancer_amd/libfd_ed25519_gpu.so || echo build/$1/libfd_ed25519_gpu.so; }
for v in $2; do
  [ "$v" = main ] && continue
  echo "[$(date +%T)] parity $v"
  FDGPU_LIB=$(lib_of $v) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 \
    --timeout-method thread > $o/tests_$v.log 2>&1 || { tail -30 $o/tests_$v.log; exit 1; }
  tail -1 $o/tests_$v.log
done
for rep in 1 2; do
  for v in $2; do
    FDGPU_LIB=$(lib_of $v) timeout -k 10 200 python3 bench.py --no-extras --steps 20 --warmup 3 \
      > $o/bench_${v}_$rep.json 2> $o/bench_${v}_$rep.err || { tail $o/bench_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$o/bench_${v}_$rep.json'));print('$v rep $rep', d['ms_per_step'], 'ms/step', round(d['value']/1e6,2), 'M/s  isolated', d['roofline']['note'].split('time ')[1][:9])"
  done
done
for v in $2; do
  FDGPU_LIB=$(lib_of $v) timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_WAVES \
    -d $o/pmc_$v -o run --output-format csv -- python3 bench.py --no-extras --queues 1 --steps 3 --warmup 1 \
    > $o/pmc_$v.json 2> $o/pmc_$v.err || { tail $o/pmc_$v.err; exit 1; }
  python3 - $o/pmc_$v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(list)
per = collections.defaultdict(float)
for r in csv.DictReader(open(f)):
    if 'verify_hs' not in r['Kernel_Name']:
        continue
    per[(r['Dispatch_Id'], r['Counter_Name'])] += float(r['Counter_Value'])
for (d, n), v in per.items():
    acc[n].append(v)
print(sys.argv[1].split('/')[-1], {k: '%.4g' % sorted(v)[len(v) // 2] for k, v in acc.items()})
PY
done
echo "[$(date +%T)] done"
