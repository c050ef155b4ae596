"""How many verify kernels the MI355X runs at once from separate streams:
N device-resident cfg1 batches of B signatures, each on its own HIP stream
and workspace (DeviceBatch.own_queue), R verifies queued on every stream
round robin from one host thread, then one device sync.  Prints the
aggregate sigs/s for each (N, B): if it stops growing with N well before N
batches fill the chip's wave slots (8 x 16 K), streams, not CUs, bound the
tiles' gathered pipeline.

    python tools/conc_probe.py [--ns 1,2,4,8,12,16] [--batches 16384] [--reps 20] [--hw-queues 32]
"""
import argparse
import json
import os
import sys
import time

_hwq = [sys.argv[i + 1] for i, a in enumerate(sys.argv[:-1]) if a == "--hw-queues"]
os.environ["GPU_MAX_HW_QUEUES"] = _hwq[0] if _hwq else "32"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import firedancer_amd as fa  # noqa: E402
from firedancer_amd import workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,2,4,8,12,16")
    ap.add_argument("--batches", default="16384")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--hw-queues", type=int, default=32)
    ap.add_argument("--pair", type=int, default=0)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    ns = [int(x) for x in args.ns.split(",")]
    bsz = [int(x) for x in args.batches.split(",")]
    arena, txns, _ = workload.cfg1(max(bsz), seed=0xC0C)
    lines = []
    for B in bsz:
        eng = fa.VerifyEngine(0, max_txn=B, max_sig=B, max_arena=len(arena) + 4096, pair=bool(args.pair))
        bs = [eng.upload(arena, txns[:B]).own_queue() for _ in range(max(ns))]
        for b in bs:                                   # warm every stream (queue creation, workspace)
            b.verify()
        eng.sync()
        ref = bs[0].codes()
        for n in ns:
            t0 = time.perf_counter()
            for _ in range(args.reps):
                for b in bs[:n]:
                    b.verify()
            eng.sync()
            dt = time.perf_counter() - t0
            ok = all((b.codes() == ref).all() for b in bs[:n])
            res = {"streams": n, "batch": B, "reps": args.reps, "pair": args.pair, "hw_queues": args.hw_queues,
                   "sigs_per_s": round(n * B * args.reps / dt, 1), "ms_per_round": round(dt / args.reps * 1e3, 3),
                   "codes_equal": ok}
            print(json.dumps(res), flush=True)
            lines.append(json.dumps(res))
        for b in bs:
            b.free()
        eng.close()
    if args.out:
        with open(args.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
