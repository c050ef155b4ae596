# round-3 call: full GPU suite and smoke at the round's head
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03final; mkdir -p $o
echo "[$(date +%T)] GPU tests"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests \
  > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -1 $o/gpu_tests.log
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log | cut -c1-400
echo "[$(date +%T)] done"
