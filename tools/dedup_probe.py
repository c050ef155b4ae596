"""The dedup tile's per-frag cost on this host, alone (no GPU): the verify
tiles' outputs prefilled into L verify -> dedup links, then one sandboxed
dedup child (fdgpu_dtile_run_sandboxed, the product loop) drains them,
pinned to one core.  Reported per tcache depth: frags/s and ns per frag,
with the tcache fresh (nothing evicted yet) and in its steady state (filled
with `depth` other tags first, so every insert evicts -- a validator that
has run longer than depth frags).

    python tools/dedup_probe.py --frags 1000000 --links 2 --depths 16384,4194302 --cpu 2
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from firedancer_amd import tile, workload  # noqa: E402


def verify_outputs(n, seed):
    """n distinct verify-tile out frags ([payload][pad][fd_txn_t][u16 sz])"""
    a, t, _ = workload.cfg1(n, seed=seed)
    outs = []
    for p in workload.payloads(a, t):
        sz, raw = tile.txn_parse(p)
        if not sz:                          # (a corrupted message the verify tile would not publish)
            continue
        pad = b"\0" if len(p) & 1 else b""
        outs.append(p + pad + raw + len(p).to_bytes(2, "little"))
    return outs


def run(outs, links, depth, steady, cpu, reps):
    n = len(outs) * reps
    per = (n + links - 1) // links
    ldepth = 1 << max(10, (per - 1).bit_length())
    ins = [tile.Link(ldepth, tile.TPU_DCACHE_MTU) for _ in range(links)]
    k = 0
    for r in range(reps):                   # repeat copies a whole stream apart (dups inside the depth)
        for f in outs:
            ins[k % links].publish(f)
            k += 1
    out = tile.Link(1 << 16, tile.TPU_DCACHE_MTU)
    dt = tile.DedupTile(ins, out, tcache_depth=depth)
    fill = dt.tcache_fill(depth + 1024, seed=depth) if steady else None
    if cpu >= 0:
        os.sched_setaffinity(0, {cpu})
    t0 = time.monotonic()
    pid, stats = dt.fork_sandboxed(n, idle_s=2.0)
    _, status = os.waitpid(pid, 0)
    st = stats()
    dt.close()
    wall = st["done_ns"] * 1e-9 - t0
    return {"depth": depth, "steady": steady, "links": links, "frags": n, "exit": os.WEXITSTATUS(status),
            "frags_per_s": round(n / wall, 1), "ns_per_frag": round(wall * 1e9 / n, 1), "stats": st,
            "fill_dups": fill}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frags", type=int, default=500_000, help="distinct verified txns")
    ap.add_argument("--reps", type=int, default=2, help="the stream published this many times over")
    ap.add_argument("--links", type=int, default=2)
    ap.add_argument("--depths", default="16384,4194302")
    ap.add_argument("--cpu", type=int, default=-1)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    outs = verify_outputs(a.frags, seed=0xDED0)
    lines = []
    for d in (int(x) for x in a.depths.split(",")):
        for steady in (False, True):
            r = run(outs, a.links, d, steady, a.cpu, a.reps)
            print(json.dumps(r), flush=True)
            lines.append(r)
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(json.dumps(x) for x in lines) + "\n")


if __name__ == "__main__":
    main()
