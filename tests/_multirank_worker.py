"""Worker for tests/test_multirank.py: runs under torch.distributed.run with
gloo on CPU and exercises bench.py's rank logic (shard seeds, barrier,
max-over-ranks time, whole-job aggregation) with the CPU oracle standing in
for the GPU engine."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from firedancer_amd import workload  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def main():
    dist = bench.Dist()
    assert dist.world == 2
    cpus = dist.cpus()                       # this rank's cores (disjoint from the other rank's)
    n = 64
    arena, txns, modes = workload.cfg1(n, seed=bench.rank_seed(dist.rank), nthreads=1)
    dist.barrier()
    t0 = time.perf_counter()
    codes = orc.verify_txns(arena, txns)
    time.sleep(0.05 * (dist.rank + 1))       # uneven ranks: the slower one defines the time
    dt = time.perf_counter() - t0
    dist.barrier()
    value, dt_max = bench.aggregate(dist, int(txns["sig_cnt"].sum()), 1, dt)
    assert dt_max >= dt
    ok = int(((codes == 0) == (modes == 0)).all())
    first = int.from_bytes(arena[1:9].tobytes(), "little")
    firsts = dist.sum(first % 1000003)
    # the node-level cfg5 lines (bench.node_lines): rank 0 runs one engine
    # process per rank over shared links, the other rank waits at the barrier;
    # the CPU stand-in engine, small links
    a2, t2, m2 = workload.cfg1(400, seed=0x40DE, nthreads=1)
    node = bench.node_lines(dist, a2, t2, m2, cpus,
                            engine_cmd=[sys.executable, os.path.join(REPO, "tests", "_engine_proc_worker.py")],
                            depth_lg=(12, 12), batch=64, inflight=2)
    out = {"rank": dist.rank, "value": value, "dt_max": dt_max, "ok": ok, "firsts_sum": firsts,
           "first": first % 1000003, "cpus": cpus, "node": node}
    path = os.environ["MULTIRANK_OUT"] + f".{dist.rank}"
    json.dump(out, open(path, "w"))
    dist.close()


if __name__ == "__main__":
    main()
