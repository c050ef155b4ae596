"""Where the PCIe-inclusive (shim) path spends its time on the GPU box:
pipelined fdgpu_submit -> fdgpu_poll over host batches, staged (copied into
the engine's pinned slots) vs registered (fdgpu_host_register: DMA'd in
place), for several batch sizes / ring depths; reports sigs/s and the host
time inside submit() per batch.

    python tools/pcie_probe.py [--txns 1000000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import firedancer_amd as fa  # noqa: E402
from firedancer_amd import workload  # noqa: E402


def views_of(arena, txns, batch, copy):
    out = []
    for s in range(0, len(txns) - batch + 1, batch):
        t = txns[s:s + batch].copy()
        lo = int(t["sig_off"].min())
        hi = int((t["msg_off"] + t["msg_sz"]).max())
        for f in ("msg_off", "sig_off", "pub_off"):
            t[f] -= lo
        out.append((np.ascontiguousarray(arena[lo:hi]) if copy else arena[lo:hi], t))
    return out


def run(eng, vs, depth, rounds=2):
    sigs, t_sub = 0, 0.0
    inflight = []
    t0 = time.perf_counter()
    for i in range(len(vs) * rounds):
        a, t = vs[i % len(vs)]
        if len(inflight) == depth:
            eng.poll(inflight.pop(0), blocking=True)
        s0 = time.perf_counter()
        inflight.append(eng.submit(a, t))
        t_sub += time.perf_counter() - s0
        sigs += int(t["sig_cnt"].sum())
    for tk in inflight:
        eng.poll(tk, blocking=True)
    wall = time.perf_counter() - t0
    return sigs / wall, t_sub / (len(vs) * rounds) * 1e3


def upload_only(eng, buf, nbytes, depth, reps=40):
    """GB/s of batches with no transactions: only the arena's H2D copy runs"""
    t = np.zeros(0, dtype=fa.ed25519.TXN_DTYPE)
    inflight = []
    t0 = time.perf_counter()
    for i in range(reps):
        if len(inflight) == depth:
            eng.poll(inflight.pop(0), blocking=True)
        inflight.append(eng.submit(buf[:nbytes], t))
    for tk in inflight:
        eng.poll(tk, blocking=True)
    return nbytes * reps / (time.perf_counter() - t0) / 1e9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=1_000_000)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    arena, txns, _ = workload.cfg1(args.txns, seed=0x9C1E)
    lines = []
    eng = fa.VerifyEngine(0, max_txn=65536, ring_depth=4)
    nb = 22 << 20
    d = {"upload_only_staged_GBps": round(upload_only(eng, arena, nb, 4), 2)}
    eng.host_register(arena)
    d["upload_only_registered_GBps"] = round(upload_only(eng, arena, nb, 4), 2)
    eng.host_unregister(arena)
    eng.close()
    print(json.dumps(d), flush=True)
    lines.append(json.dumps(d))
    for batch, depth in ((65536, 4), (65536, 6), (65536, 8), (32768, 8), (131072, 6)):
        eng = fa.VerifyEngine(0, max_txn=batch, ring_depth=depth)
        staged = views_of(arena, txns, batch, True)
        r_st = run(eng, staged, depth)
        eng.host_register(arena)
        r_rg = run(eng, views_of(arena, txns, batch, False), depth)
        eng.host_unregister(arena)
        eng.close()
        d = {"batch_txns": batch, "ring_depth": depth,
             "staged_sigs_per_s": round(r_st[0], 1), "staged_submit_ms": round(r_st[1], 3),
             "registered_sigs_per_s": round(r_rg[0], 1), "registered_submit_ms": round(r_rg[1], 3),
             "arena_bytes_per_sig": round(len(arena) / len(txns), 1)}
        print(json.dumps(d), flush=True)
        lines.append(json.dumps(d))
    if args.out:
        open(args.out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
