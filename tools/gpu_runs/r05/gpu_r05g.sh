set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 5 60 tools/ubench_pcie > $O/ubench_pcie.jsonl 2>&1; cat $O/ubench_pcie.jsonl
FE=build/feasm/libfd_ed25519_gpu.so
timeout -k 10 300 env FDGPU_LIB=$FE python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/feasm_parity.log 2>&1 || { echo FEASM_PARITY_FAILED; tail -20 $O/feasm_parity.log; exit 1; }
tail -2 $O/feasm_parity.log
for i in 1 2; do
  timeout -k 10 120 python -u bench.py --no-extras --steps 30 --warmup 5 > $O/base_$i.json 2>$O/base_$i.err || { echo BASE_FAILED; tail $O/base_$i.err; exit 1; }
  timeout -k 10 120 env FDGPU_LIB=$FE python -u bench.py --no-extras --steps 30 --warmup 5 > $O/feasm_$i.json 2>$O/feasm_$i.err || { echo FEASM_FAILED; tail $O/feasm_$i.err; exit 1; }
  python -c "
import json
for t in ('base_$i','feasm_$i'):
  d=json.loads(open('$O/'+t+'.json').read().strip().splitlines()[-1]); print(t, d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
