# Table-read traffic A/B, second pass: pad64 = entries padded to 256 B (correct codes); line8 = pad64 staging
# one 128-B line per entry (wrong codes: the traffic of a packed entry).  First pass:: base vs FDGPU_DIAG_TAB_HOT (chain table
# reads turned into L2 hits, same VALU work, wrong codes -> bench exits 3 after its line)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05tab2; mkdir -p $O
export TMPDIR=/tmp
ok() { [ $1 -eq 0 ] || { [ $2 = line8 ] && [ $1 -eq 3 ]; }; }
for v in "pad64::build/pad64/libfd_ed25519_gpu.so" "line8::build/line8/libfd_ed25519_gpu.so"; do
  tag=${v%%::*}; lib=${v#*::}
  p=0
  for CTR in "SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" "FETCH_SIZE"; do
    p=$((p+1))
    FDGPU_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $CTR -d $O/pmc_${tag}_$p -o run --output-format csv -- python3 bench.py --no-extras --queues 1 --steps 3 --warmup 1 > $O/pmc_${tag}_$p.json 2>$O/pmc_${tag}_$p.err
    rc=$?; ok $rc $tag || { echo PMC_FAILED $tag $p rc=$rc; tail $O/pmc_${tag}_$p.err; exit 1; }
    python3 tools/pmc_kernel.py fdgpu_verify_hs_kernel $(find $O/pmc_${tag}_$p -name "*counter_collection.csv") > $O/verify_${tag}_$p.json || exit 1
  done
done
for i in 1 2; do for v in "base::firedancer_amd/libfd_ed25519_gpu.so" "pad64::build/pad64/libfd_ed25519_gpu.so" "line8::build/line8/libfd_ed25519_gpu.so"; do
  tag=${v%%::*}; lib=${v#*::}
  FDGPU_LIB=$lib timeout -k 10 120 python3 bench.py --no-extras --steps 30 --warmup 5 > $O/time_${tag}_$i.json 2>$O/time_${tag}_$i.err
  rc=$?; ok $rc $tag || { echo TIME_FAILED $tag rc=$rc; tail $O/time_${tag}_$i.err; exit 1; }
done; done
python3 - <<PY
import json
for t in ('base','pad64','line8'):
    d={}
    for p in ((1,2) if t!='base' else ()): d.update(json.load(open('$O/verify_%s_%d.json'%(t,p))))
    print(t, {k: '%.4g'%v for k,v in d.items()})
    for i in (1,2):
        b=json.load(open('$O/time_%s_%d.json'%(t,i))); print('  ', b['value'], b['ms_per_step'], b['roofline']['frac'], b.get('parity_mismatches'))
PY
