set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05v; mkdir -p $O
export TMPDIR=/tmp
CTR="SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for v in "base::firedancer_amd/libfd_ed25519_gpu.so" "feasm::build/feasm/libfd_ed25519_gpu.so"; do
  tag=${v%%::*}; lib=${v#*::}
  FDGPU_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $CTR -d $O/pmc_$tag -o run --output-format csv -- python3 bench.py --no-extras --queues 1 --steps 3 --warmup 1 > $O/pmc_$tag.json 2>$O/pmc_$tag.err || { echo PMC_FAILED $tag; tail $O/pmc_$tag.err; exit 1; }
  python3 tools/pmc_kernel.py fdgpu_verify_hs_kernel $(find $O/pmc_$tag -name "*counter_collection.csv") > $O/verify_$tag.json || exit 1
done
for i in 1 2; do for v in "base::firedancer_amd/libfd_ed25519_gpu.so" "feasm::build/feasm/libfd_ed25519_gpu.so"; do
  tag=${v%%::*}; lib=${v#*::}
  FDGPU_LIB=$lib timeout -k 10 120 python3 bench.py --no-extras --steps 30 --warmup 5 > $O/time_${tag}_$i.json 2>$O/time_${tag}_$i.err || { echo TIME_FAILED $tag; tail $O/time_${tag}_$i.err; exit 1; }
done; done
python3 -c "
import json
for t in ('base','feasm'):
    d=json.load(open('$O/verify_'+t+'.json')); print(t, {k: '%.4g'%v for k,v in d.items()})
    for i in (1,2):
        b=json.load(open('$O/time_%s_%d.json'%(t,i))); print('  ', b['value'], b['roofline']['frac'])
"
