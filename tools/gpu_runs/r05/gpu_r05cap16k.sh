# Tile throughput at the reference's link depth: paced runs offered more than the
# tiles can take, on 16,384-deep quic->verify links (default.toml receive_buffer_size), lap guard on.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05cap16k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/make_tile_npz.py --out /tmp/cfg1.npz > $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --payload-npz /tmp/cfg1.npz --depth-lg 21 --depth-lg-paced 14 --paced-reps 4 --pair 2 --spread 2 --wait-us 200 --reps 2 --hw-queues 32 --pin 1"
for sw in "1,16384,8,24e6,2" "1,16384,8,36e6,3" "1,16384,8,48e6,4" "2,16384,8,36e6,4" "2,16384,8,48e6,4" "2,16384,8,60e6,6" "2,16384,8,72e6,6"; do
  timeout -k 10 170 python -u tools/bench_tile.py $C --sweep "$sw" --out $O/x.jsonl >> $O/x.log 2>&1
  rc=$?; [ $rc -le 1 ] || { echo RUN_FAILED $sw rc $rc; tail -5 $O/x.log; exit 1; }   # 1: a run lost frags (expected here)
done
grep '^{"metric"' $O/x.log | python -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l); c=d['counters']; print(d['tiles'], d['producers'], d['rate_target']/1e6, round((d.get('offered_txns_per_s') or 0)/1e6,1), round(d['txns_per_s']/1e6,2), d['batch_latency_ms'], 'overrun', c['overrun'], 'lapped', c['lapped'], 'rescued', c['rescued'], 'ok', d['published_ok'])
"
