# round-3 call: headline step time vs overlapped device-resident copies (queues)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03z; mkdir -p $o
for q in 2 3 4 2; do
  echo "[$(date +%T)] queues $q"
  timeout -k 10 300 python3 bench.py --no-extras --queues $q --steps 30 --warmup 3 > $o/q$q.json 2> $o/q$q.err || { tail $o/q$q.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$o/q$q.json').read().strip().splitlines()[-1]); print(' value', d['value'], 'ms', d['ms_per_step'])"
done
echo "[$(date +%T)] done"
