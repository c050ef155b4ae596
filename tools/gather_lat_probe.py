"""The gathered-frag batch latency line of bench.py (latency_frag_io) on its
own, for a kernel trace: one engine, cfg1 frags, `--batches` batches of
`--batch` frags, one in flight; prints the bench's p50/p99 fields and the
per-batch latencies (ms, in order) to --out so a trace's slow batches can
be matched to them.

    python tools/gather_lat_probe.py [--batch 65536] [--batches 1000] [--out f.json]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

import bench  # noqa: E402
import firedancer_amd as fa  # noqa: E402
from firedancer_amd import workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--batches", type=int, default=1000)
    ap.add_argument("--pin", type=int, default=1)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    arena, txns, _ = workload.cfg1(args.batch * 4, seed=0x1A7)
    eng = fa.VerifyEngine(0, max_txn=len(txns), max_sig=len(txns) * 12, max_arena=len(arena) + 4096, ring_depth=2)
    ref = eng.verify_txns(arena, txns)
    res = bench.latency_frag_io(eng, arena, txns, ref, args.batch, args.batches,
                                pin_cpu=workload.physical_cpus()[1] if args.pin else None, keep_raw=True)
    print(json.dumps({k: v for k, v in res.items() if k != "lat_ms"}), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f)
    eng.close()


if __name__ == "__main__":
    main()
