"""The gathered-frag GPU pipeline's own capacity, without a tile: E engines
(one per would-be tile) each keep K batches of B cfg1 frags in flight
through fdgpu_submit_frags_io / fdgpu_poll_frags_io, from one host thread,
resubmitting the same registered frags as soon as a batch completes.  Gives
txn/s for each (E, K, B) -- the ceiling the mux tiles' end-to-end rate can
reach on this box -- and the mean per-batch time submit -> completion.

    python3 tools/pipe_conc.py --runs "1,4,16384;2,4,16384;2,8,8192" --batches 200
"""
import argparse
import json
import os
import sys
import time

# the box exports GPU_MAX_HW_QUEUES=4; --hw-queues N (default 32) must win, before HIP starts
_hwq = [a.split("=", 1)[1] if "=" in a else None for a in sys.argv if a.startswith("--hw-queues")]
os.environ["GPU_MAX_HW_QUEUES"] = (_hwq[0] if _hwq and _hwq[0] else
                                   (sys.argv[sys.argv.index("--hw-queues") + 1] if "--hw-queues" in sys.argv else "32"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from firedancer_amd import _lib, tile, workload  # noqa: E402
import firedancer_amd as fa  # noqa: E402
from firedancer_amd.ed25519 import FRAG_IO_DTYPE  # noqa: E402


def frag_batch(B, seed=5):
    a, t, _ = workload.cfg1(B, seed=seed)
    ps = workload.payloads(a, t)
    L = _lib.lib()
    src = np.zeros(B * 1280 + 8192, dtype=np.uint8)
    src = src[(-src.ctypes.data) % 4096:][:B * 1280 + 4096]
    caps = [L.fdgpu_frag_out_cap(len(p)) for p in ps]
    out_bytes = sum((c + 63) // 64 * 64 for c in caps)
    out = np.zeros(out_bytes + 8192, dtype=np.uint8)
    out = out[(-out.ctypes.data) % 4096:][:out_bytes + 4096]
    fio = np.zeros(B, dtype=FRAG_IO_DTYPE)
    o = 0
    for k, p in enumerate(ps):
        src[k * 1280:k * 1280 + len(p)] = np.frombuffer(p, dtype=np.uint8)
        fio[k] = (src.ctypes.data + k * 1280, len(p), o, caps[k], 0, 0)
        o += (caps[k] + 63) // 64 * 64
    return src, out, out_bytes, fio


def run(E, K, B, batches):
    engines = [fa.VerifyEngine(0, max_txn=B, max_sig=B * 12, max_arena=B * 1280, ring_depth=K) for _ in range(E)]
    bufs = [frag_batch(B, seed=5 + k) for k in range(E)]
    for e, (src, out, ob, fio) in zip(engines, bufs):
        e.host_register(src)
        e.host_register(out)
        for tk in [e.submit_frags_io(fio, out, ob, 1) for _ in range(K)]:      # warm every slot
            e.poll_frags_io(tk, blocking=True)
    codes = np.zeros(B, dtype=np.int8)
    tags = np.zeros(B, dtype=np.uint64)
    szs = np.zeros(B, dtype=np.uint16)
    L = _lib.lib()
    fl = [[] for _ in range(E)]
    done = submitted = 0
    span = 0.0
    t0 = time.perf_counter()
    while done < batches:
        for k, e in enumerate(engines):
            src, out, ob, fio = bufs[k]
            while len(fl[k]) < K and submitted < batches:
                fl[k].append((e.submit_frags_io(fio, out, ob, 1), time.perf_counter()))
                submitted += 1
            if fl[k]:
                tk, ts = fl[k][0]
                rc = L.fdgpu_poll_frags_io(e._h, tk, codes.ctypes.data, tags.ctypes.data, szs.ctypes.data, 0)
                if rc == 0:
                    fl[k].pop(0)
                    done += 1
                    span += time.perf_counter() - ts
                elif rc != 1:
                    raise SystemExit(f"poll rc {rc}")
    wall = time.perf_counter() - t0
    for e, (src, out, _, _) in zip(engines, bufs):
        e.host_unregister(src)
        e.host_unregister(out)
        e.close()
    return {"engines": E, "inflight": K, "batch": B, "batches": batches,
            "txns_per_s": round(batches * B / wall, 1), "batch_ms": round(span / batches * 1e3, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", default="1,4,16384;2,4,16384;2,8,8192;2,8,16384;4,4,16384")
    ap.add_argument("--batches", type=int, default=200)
    ap.add_argument("--out", default="")
    ap.add_argument("--hw-queues", type=int, default=32, help="GPU_MAX_HW_QUEUES (set before HIP initialises)")
    args = ap.parse_args()
    for r in args.runs.split(";"):
        E, K, B = (int(x) for x in r.split(","))
        res = run(E, K, B, args.batches)
        res["hw_queues"] = int(os.environ["GPU_MAX_HW_QUEUES"])
        print(json.dumps(res), flush=True)
        if args.out:
            with open(args.out, "a") as f:
                f.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
