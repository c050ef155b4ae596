"""Batch latency / PCIe-inclusive throughput sweep over batch size, ring depth
and sub-batch split (one logical batch spread over several ring slots, whose
streams overlap copy and compute).  One JSON line per configuration.

    python tools/latency_sweep.py --txns 262144 --batches 8192,16384,65536 --depths 2,4 --splits 1,2,4
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def views_of(arena, txns, batch):
    out = []
    for s in range(0, len(txns) - batch + 1, batch):
        t = txns[s:s + batch].copy()
        lo = int(t["sig_off"].min())
        hi = int((t["msg_off"] + t["msg_sz"]).max())
        for f in ("msg_off", "sig_off", "pub_off"):
            t[f] -= lo
        out.append((np.ascontiguousarray(arena[lo:hi]), t))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=262144)
    ap.add_argument("--batches", default="8192,16384,32768,65536")
    ap.add_argument("--depths", default="2,4")
    ap.add_argument("--splits", default="1,2,4")
    ap.add_argument("--reps", type=int, default=100)
    a = ap.parse_args()
    from firedancer_amd import VerifyEngine, workload
    arena, txns, _ = workload.cfg1(a.txns, seed=7)
    src = arena[:16 << 20].copy()
    dst = np.empty_like(src)
    t0 = time.perf_counter()
    for _ in range(20):
        np.copyto(dst, src)
    print(json.dumps({"numpy_memcpy_GBps": round(20 * src.size / (time.perf_counter() - t0) / 1e9, 2)}), flush=True)
    for depth in [int(x) for x in a.depths.split(",")]:
        for batch in [int(x) for x in a.batches.split(",")]:
            for split in [int(x) for x in a.splits.split(",")]:
                if split > depth or batch % split:
                    continue
                sub = batch // split
                eng = VerifyEngine(0, max_txn=sub, max_sig=2 * sub, max_arena=sub * 1232, ring_depth=depth)
                vs = views_of(arena, txns, sub)
                for i in range(10):
                    eng.verify_txns(*vs[i % len(vs)])
                lat, lsub = [], []
                for r in range(a.reps):
                    t0 = time.perf_counter()
                    tks = [eng.submit(*vs[(r * split + j) % len(vs)]) for j in range(split)]
                    lsub.append((time.perf_counter() - t0) * 1e3)
                    for tk in tks:
                        eng.poll(tk, blocking=True)
                    lat.append((time.perf_counter() - t0) * 1e3)
                sigs, inflight, t_sub, nsub = 0, [], 0.0, 0
                t0 = time.perf_counter()
                for i in range(max(len(vs), 4 * depth) * 2):
                    if len(inflight) == depth:
                        eng.poll(inflight.pop(0), blocking=True)
                    av, tv = vs[i % len(vs)]
                    ts = time.perf_counter()
                    inflight.append(eng.submit(av, tv))
                    t_sub += time.perf_counter() - ts
                    nsub += 1
                    sigs += int(tv["sig_cnt"].sum())
                for tk in inflight:
                    eng.poll(tk, blocking=True)
                rate = sigs / (time.perf_counter() - t0)
                eng.close()
                lat = np.array(lat)
                print(json.dumps({"batch": batch, "split": split, "ring_depth": depth,
                                  "p50_ms": round(float(np.percentile(lat, 50)), 3),
                                  "p99_ms": round(float(np.percentile(lat, 99)), 3),
                                  "pipelined_sigs_per_s": round(rate, 1),
                                  "submit_host_ms": round(t_sub / nsub * 1e3, 3),
                                  "submit_idle_ms": round(float(np.median(lsub)), 3),
                                  "submit_idle_p99_ms": round(float(np.percentile(lsub, 99)), 3),
                                  "p999_ms": round(float(np.percentile(lat, 99.9)), 3),
                                  "n_over_2x_p50": int((lat > 2 * np.percentile(lat, 50)).sum()),
                                  "arena_mb": round(sum(v[0].size for v in vs) / len(vs) / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
