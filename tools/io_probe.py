"""Gathered-batch engine capacity with no tile around it: E engines, each
driven by a host thread that keeps `inflight` fdgpu_submit_frags_io batches of
`batch` frags in flight (payloads in a registered in buffer at 64-B chunk
offsets, out frags into a registered out buffer), polling the oldest.  Tells
the device side of the gathered path (ingest + verify + finish) apart from
the mux tile's host loop.

    python tools/io_probe.py --npz /tmp/cfg1.npz --engines 2 --batch 16384 --inflight 8 [--out f.jsonl]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import _lib  # noqa: E402
from firedancer_amd.ed25519 import FRAG_IO_DTYPE, VerifyEngine  # noqa: E402


def aligned(n):
    raw = np.zeros(n + 4096, dtype=np.uint8)
    a = (-raw.ctypes.data) % 4096
    return raw[a:a + n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npz", required=True)
    ap.add_argument("--engines", type=int, default=1)
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--inflight", type=int, default=8)
    ap.add_argument("--batches", type=int, default=64, help="timed batches per engine")
    ap.add_argument("--pair", type=int, default=2)
    ap.add_argument("--spread", type=int, default=2)
    ap.add_argument("--tag", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    z = np.load(a.npz)
    arena, offs, sizes = z["arena"], z["offs"], z["sizes"]
    L = _lib.lib()
    n_per = a.batch * a.inflight                 # distinct batches per engine (reused round robin)
    res = []
    engines = [VerifyEngine(0, max_txn=a.batch, max_arena=a.batch * 1232, ring_depth=a.inflight,
                            pair=a.pair == 1, pair_auto=a.pair == 2, spread=a.spread == 1, spread_auto=a.spread == 2)
               for _ in range(a.engines)]
    bufs = []
    for ei, eng in enumerate(engines):
        eng.reserve()
        idx = (np.arange(n_per) + ei * n_per) % len(offs)
        sz = sizes[idx].astype(np.int64)
        chunk = (sz + 63) // 64 * 64
        ioff = np.concatenate([[0], np.cumsum(chunk)[:-1]])
        inb = aligned(int(chunk.sum()) + 4096)
        for k in range(n_per):                                  # payloads into the "in dcache"
            o = int(offs[idx[k]])
            inb[ioff[k]:ioff[k] + sz[k]] = arena[o:o + sz[k]]
        cap = np.array([L.fdgpu_frag_out_cap(int(s)) for s in sz], dtype=np.int64)
        ocap = (cap + 63) // 64 * 64
        outb = aligned(int(ocap.reshape(a.inflight, a.batch).sum(axis=1).max()) * a.inflight + 4096)
        eng.host_register(inb)
        eng.host_register(outb)
        fios, views = [], []
        obase = 0
        for b in range(a.inflight):
            sl = slice(b * a.batch, (b + 1) * a.batch)
            fio = np.zeros(a.batch, dtype=FRAG_IO_DTYPE)
            oo = np.concatenate([[0], np.cumsum(ocap[sl])[:-1]])
            fio["src"] = inb.ctypes.data + ioff[sl]
            fio["sz"] = sz[sl]
            fio["out_off"] = oo
            fio["out_cap"] = cap[sl]
            osz = int(ocap[sl].sum())
            fios.append(fio)
            views.append((outb[obase:obase + osz], osz))
            obase += osz
        bufs.append((inb, outb, fios, views))

    def drive(ei, n_batches, lat):
        eng = engines[ei]
        _, _, fios, views = bufs[ei]
        q = []
        for i in range(n_batches):
            if len(q) == a.inflight:
                tk, t0 = q.pop(0)
                eng.poll_frags_io(tk)
                lat.append(time.perf_counter() - t0)
            b = i % a.inflight
            q.append((eng.submit_frags_io(fios[b], views[b][0], views[b][1], 0x5EED), time.perf_counter()))
        for tk, t0 in q:
            eng.poll_frags_io(tk)
            lat.append(time.perf_counter() - t0)

    for ei in range(a.engines):                                  # warm
        drive(ei, a.inflight * 2, [])
    lats = [[] for _ in engines]
    ths = [threading.Thread(target=drive, args=(ei, a.batches, lats[ei])) for ei in range(a.engines)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    wall = time.perf_counter() - t0
    lat = np.array(sum(lats, [])) * 1e3
    r = {"tag": a.tag, "engines": a.engines, "batch": a.batch, "inflight": a.inflight, "pair": a.pair,
         "spread": a.spread, "io_dma": os.environ.get("FDGPU_IO_DMA", "0"),
         "txns_per_s": a.engines * a.batches * a.batch / wall, "wall_s": round(wall, 4),
         "batch_latency_ms": {"p50": round(float(np.percentile(lat, 50)), 3),
                              "p99": round(float(np.percentile(lat, 99)), 3)}}
    print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "a") as f:
            f.write(json.dumps(r) + "\n")
    for eng, (inb, outb, _, _) in zip(engines, bufs):
        eng.host_unregister(inb)
        eng.host_unregister(outb)
        eng.close()


if __name__ == "__main__":
    main()
