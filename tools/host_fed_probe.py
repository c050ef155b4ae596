"""Host-fed verify at the headline size (bench.py host_fed) with its knobs
exposed, for A/Bs and rocprofv3 traces: 1M cfg2 txns per batch fed from
host memory through fdgpu_submit with --ring slots; --feed registered (DMA
straight from the arena, fdgpu_host_register) or staged (copied into pinned
slots); --arena-pages thp puts the host arena on 2 MB pages.

    python tools/host_fed_probe.py --ring 3 --feed registered --steps 12
"""
import argparse
import json
import mmap
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from firedancer_amd import VerifyEngine, _lib, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=1_000_000)
    ap.add_argument("--ring", default="3", help="ring slots; ','-separated for several runs")
    ap.add_argument("--feed", default="registered,staged")
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--arena-pages", default="4k", help="4k, thp, or both ('4k,thp')")
    ap.add_argument("--reps", type=int, default=1)
    a = ap.parse_args()
    arena0, txns, _ = workload.cfg1(a.txns, seed=workload.CFG1_SEED)
    n_sig = int(txns["sig_cnt"].sum())
    L = _lib.lib()
    for pages in a.arena_pages.split(","):
        if pages == "thp":
            sz = (arena0.nbytes + (4 << 20) + (2 << 20) - 1) // (2 << 20) * (2 << 20)
            mm = mmap.mmap(-1, sz, mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
            raw = np.frombuffer(mm, dtype=np.uint8)
            off = (-raw.ctypes.data) % (2 << 20)
            mm.madvise(mmap.MADV_HUGEPAGE, off, sz - (2 << 20))
            arena = raw[off:off + arena0.nbytes]
            arena[:] = arena0
        else:
            arena = np.ascontiguousarray(arena0)
        for ring in (int(x) for x in a.ring.split(",")):
            run(a, L, arena, txns, n_sig, ring, pages)


def run(a, L, arena, txns, n_sig, ring, pages):
    eng = VerifyEngine(0, max_txn=len(txns), max_sig=n_sig, max_arena=arena.nbytes, ring_depth=ring)
    ref = eng.verify_txns(arena, txns)
    for feed in a.feed.split(","):
        if feed == "registered":
            eng.host_register(arena)
        for rep in range(a.reps):
            tks = [eng.submit(arena, txns) for _ in range(ring)]
            for tk in tks:
                eng.poll(tk)
            tks = []
            t0 = time.perf_counter()
            for _ in range(a.steps):
                if len(tks) == ring:
                    last = eng.poll(tks.pop(0))
                tks.append(eng.submit(arena, txns))
            for tk in tks:
                last = eng.poll(tk)
            dt = time.perf_counter() - t0
            out = np.zeros(3 * a.steps, dtype=np.uint64)
            n = int(L.fdgpu_debug_submit_times(out.ctypes.data, a.steps))
            parts = (out[:3 * n].reshape(n, 3) / 1e6).mean(axis=0).round(3).tolist()
            print(json.dumps({"feed": feed, "ring": ring, "arena_pages": pages, "rep": rep,
                              "sigs_per_s": round(a.steps * n_sig / dt, 1), "ms_per_batch": round(dt / a.steps * 1e3, 3),
                              "submit_stage_expand_enqueue_ms": parts, "codes_equal": bool((last == ref).all()),
                              "h2d_link_gbps": round(L.fdgpu_debug_h2d_gbps(eng._h, arena.ctypes.data,
                                                                            256 << 20, 10), 2)
                              if feed == "registered" else None}), flush=True)
        if feed == "registered":
            eng.host_unregister(arena)
    eng.close()


if __name__ == "__main__":
    main()
