# round-3 call: the driver's GPU suite and smoke at HEAD
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03i; mkdir -p $o
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -3 $o/smoke.log
echo "[$(date +%T)] done"
