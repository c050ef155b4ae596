"""The QUIC tiles' side of the quic -> verify links, as a process of its own
(test and bench infrastructure: the QUIC tile is out of scope, SURVEY.md
§2.3).  Joins each link by path (tile.Link.shm_join) and publishes frags
into it from one C producer thread per link (fdgpu_producer_start: payload
into the compact dcache, then the mcache line, no backpressure -- the
reference's quic -> verify links are unreliable, fd_frankendancer.c:131-133).
No GPU is touched here.

Feeds (as tools/bench_tile.py deals them): "paced" -- link j carries every
P-th frag of the payload list, the list published --reps times over, at
--rate frags/s in total; "prefill" -- every link carries the whole list
(link j starting a j/P-th of the way in), published as fast as possible.

    python tools/quic_feed.py --link /dev/shm/qv0 --link /dev/shm/qv1 \\
        --npz frags.npz --mode paced --rate 16e6 --reps 4 --cpus 3,4 \\
        [--wait-file F] --result feed.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from firedancer_amd import tile  # noqa: E402


def feeds(offs, sizes, P, mode, reps):
    """(offs, sizes) per link"""
    if mode == "prefill":
        n = len(offs)
        return [(np.roll(offs, -(j * n // P)), np.roll(sizes, -(j * n // P))) for j in range(P)]
    return [(np.tile(offs[j::P], reps), np.tile(sizes[j::P], reps)) for j in range(P)]


def frag_counts(n, P, mode, reps):
    """frags each link will carry (the engine process's --frags)"""
    if mode == "prefill":
        return [n] * P
    return [len(range(j, n, P)) * reps for j in range(P)]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--link", action="append", required=True)
    ap.add_argument("--npz", required=True, help="arena, offs, sizes (bench_tile's payload file)")
    ap.add_argument("--mode", choices=("paced", "prefill"), default="paced")
    ap.add_argument("--rate", type=float, default=0.0, help="paced: frags/s over all links (0: unpaced)")
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--cpus", default="", help="producer j pinned to the j-th CPU")
    ap.add_argument("--wait-file", action="append", default=[],
                    help="start publishing once this file exists (repeat: once all of them exist)")
    ap.add_argument("--timeout", type=float, default=120.0)
    ap.add_argument("--result", default="")
    a = ap.parse_args(argv)
    z = np.load(a.npz)
    arena, offs, sizes = z["arena"], z["offs"].astype(np.uint64), z["sizes"].astype(np.uint32)
    links = [tile.Link.shm_join(p) for p in a.link]
    P = len(links)
    fd = feeds(offs, sizes, P, a.mode, a.reps)
    cpus = [int(x) for x in a.cpus.split(",") if x]
    t0 = time.monotonic()
    for wf in a.wait_file:
        while not os.path.exists(wf):
            if time.monotonic() - t0 > a.timeout:
                raise SystemExit("quic_feed: timed out waiting for " + wf)
            time.sleep(0.0005)
    keep = os.sched_getaffinity(0)
    prods = []
    t_start = time.monotonic()
    for j, ln in enumerate(links):
        if cpus:
            os.sched_setaffinity(0, {cpus[j % len(cpus)]})          # the C thread inherits the mask
        rate = 0.0 if a.mode == "prefill" else a.rate / P
        prods.append(tile.Producer(ln, arena, fd[j][0], fd[j][1], rate_tps=rate))
    os.sched_setaffinity(0, keep)
    joined = [p.join() for p in prods]
    t_end = time.monotonic()
    res = {"pid": os.getpid(), "links": P, "mode": a.mode, "rate": a.rate, "reps": a.reps,
           "published": [int(n) for n, _ in joined], "producer_s": [round(s, 6) for _, s in joined],
           "t_start": t_start, "t_end": t_end,
           "offered_per_s": round(sum(n for n, _ in joined) / max(s for _, s in joined), 1)
           if max(s for _, s in joined) > 0 else None,
           "huge_bytes": [ln.huge_bytes() for ln in links]}
    line = json.dumps(res)
    if a.result:
        with open(a.result + ".tmp", "w") as f:
            f.write(line + "\n")
        os.rename(a.result + ".tmp", a.result)
    print(line, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
