"""Host-thread scaling of the async batch API on one MI355X: T threads, each
with its own engine (as bench_tile gives each verify tile), each keeping
`inflight` batches of `batch` cfg1 txns in flight (submit -> poll).  Reports
per-thread and aggregate sigs/s and the mean submit->poll latency, so the
GPU/runtime side of the tile's multi-thread scaling is seen without the
tango ingest.

    python tools/engine_mt_probe.py --threads 1,2,4 --batch 16384 --inflight 4
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import firedancer_amd as fa  # noqa: E402
from firedancer_amd import workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,2,4")
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--inflight", type=int, default=4)
    ap.add_argument("--iters", type=int, default=64, help="batches per thread")
    ap.add_argument("--shared", type=int, default=0, help="1: all threads share one engine")
    args = ap.parse_args()
    arena, txns, _ = workload.cfg1(args.batch, seed=11)
    for T in [int(x) for x in args.threads.split(",")]:
        ne = 1 if args.shared else T
        engines = [fa.VerifyEngine(0, max_txn=args.batch, max_arena=args.batch * 1232,
                                   ring_depth=args.inflight * (T if args.shared else 1)) for _ in range(ne)]
        for e in engines:                       # first use of every slot's stream
            tks = [e.submit(arena, txns) for _ in range(e_depth(args, T))]
            for tk in tks:
                e.poll(tk, blocking=True)
        lat = [[] for _ in range(T)]
        barrier = threading.Barrier(T + 1)

        def body(k):
            e = engines[0 if args.shared else k]
            barrier.wait()
            q = []
            for i in range(args.iters):
                if len(q) == args.inflight:
                    tk, t0 = q.pop(0)
                    e.poll(tk, blocking=True)
                    lat[k].append(time.perf_counter() - t0)
                q.append((e.submit(arena, txns), time.perf_counter()))
            for tk, t0 in q:
                e.poll(tk, blocking=True)
                lat[k].append(time.perf_counter() - t0)
        ths = [threading.Thread(target=body, args=(k,)) for k in range(T)]
        for th in ths:
            th.start()
        barrier.wait()
        t0 = time.perf_counter()
        for th in ths:
            th.join()
        wall = time.perf_counter() - t0
        sigs = T * args.iters * len(txns)
        print(json.dumps({"threads": T, "shared_engine": bool(args.shared), "batch": args.batch,
                          "inflight": args.inflight, "sigs_per_s": round(sigs / wall, 1), "wall_s": round(wall, 4),
                          "lat_ms_mean": round(1e3 * float(np.mean(np.concatenate([np.array(x) for x in lat]))), 3)}),
              flush=True)
        for e in engines:
            e.close()


def e_depth(args, T):
    return args.inflight * (T if args.shared else 1)


if __name__ == "__main__":
    main()
