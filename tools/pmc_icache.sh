set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/ic; mkdir -p $o
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_MISSES -d $o/p0 -o run --output-format csv -- python3 bench.py --no-extras --queues 1 --steps 3 --warmup 1 > $o/p0.json 2> $o/p0.err || { tail $o/p0.err; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQ_IFETCH -d $o/p1 -o run --output-format csv -- python3 bench.py --no-extras --queues 1 --steps 3 --warmup 1 > $o/p1.json 2> $o/p1.err || { tail $o/p1.err; exit 1; }
echo done
