set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05u; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/make_tile_npz.py --multi 1 --out /tmp/cfg3.npz >> $O/npz.log 2>&1 || { echo NPZ_FAILED; tail $O/npz.log; exit 1; }
C="--mux 1 --gpu-parse 2 --depth-lg 21 --depth-lg-paced 14 --paced-reps 4 --pair 2 --spread 2 --wait-us 200 --reps 3 --hw-queues 32 --producers-same-as-tiles 1 --multi 1 --batch-sig-max 24576 --payload-npz /tmp/cfg3.npz"
for sw in "1,16384,8,-1,1,24576;2,16384,8,-1,2,24576" "2,16384,8,-1,2,32768" "2,16384,8,-1,2,49152" "1,16384,8,-1,1,32768" "2,16384,6,-1,2,32768"; do
  timeout -k 10 170 python -u tools/bench_tile.py $C --sweep "$sw" --out $O/cfg3.jsonl >> $O/cfg3.log 2>&1 || { echo RUN_FAILED $sw; tail -5 $O/cfg3.log; exit 1; }
done
python -c "
import json
for l in open('$O/cfg3.jsonl'):
    d=json.loads(l); print(d['tiles'], d['inflight'], d.get('batch_sig_max'), round(d['txns_per_s']/1e6,2), round(d['sigs_per_s']/1e6,2), d['batch_latency_ms'], d['published_ok'])
"
