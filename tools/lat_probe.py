"""Batch-latency tails vs where the submitting thread runs: bench.py's
latency loops (65,536-txn batches, one in flight) repeated with the thread
pinned to each CPU given, or unpinned ("-").  Prints p50/p99 of the staged
and registered loops and the submit / rest split for each.

    python3 tools/lat_probe.py --pins "0,1,8,-" --batches 1000
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402  (sets GPU_MAX_HW_QUEUES before HIP starts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pins", default="0,1,-")
    ap.add_argument("--batches", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--txns", type=int, default=1_000_000)
    args = ap.parse_args()
    from firedancer_amd import VerifyEngine, workload
    arena, txns, _ = workload.cfg1(args.txns, seed=bench.rank_seed(0))
    eng = VerifyEngine(0, max_txn=args.batch, max_sig=2 * args.batch, max_arena=args.batch * 1232,
                       ring_depth=bench.RING_DEPTH)
    for p in args.pins.split(","):
        pin = None if p == "-" else int(p)
        r = bench.latency_and_pcie(eng, arena, txns, args.batch, args.batches, pin_cpu=pin)
        out = {"pin": p, **{k: v for k, v in r.items() if "latency" in k}}
        print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
