"""GPU-side ingest on its own, for rocprofv3 (kernel trace / PMC passes):
the cfg2 batch (1M single-signature txns) as raw payloads in a frag batch,
verified `--iters` times (parse -> scan -> expand -> verify -> combine each
time), then the HIP-event split of one pass.

    python tools/ingest_probe.py [--txns 1000000] [--iters 3]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from firedancer_amd import VerifyEngine, workload  # noqa: E402
from firedancer_amd.ed25519 import FRAG_DTYPE  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    arena, txns, _ = workload.cfg1(args.txns, seed=workload.CFG1_SEED)
    frags = np.zeros(len(txns), dtype=FRAG_DTYPE)
    frags["off"] = txns["sig_off"] - 1
    frags["sz"] = txns["msg_off"] + txns["msg_sz"] - frags["off"]
    eng = VerifyEngine(0)
    fb = eng.upload_frags(arena, frags)
    for _ in range(args.iters):
        fb.verify()
    codes = fb.codes()
    _, tsz = fb.txns(records=False)
    wall, ing, ver, comb = fb.time2(args.iters)
    n_sig = fb.n_sig
    ing_bytes = int(frags["sz"].sum()) + int(tsz.sum()) + len(frags) * 50 + n_sig * 16
    print(json.dumps({"txns": len(txns), "sigs": n_sig, "parsed": int((tsz > 0).sum()),
                      "ingest_ms": round(ing, 4), "verify_ms": round(ver, 4), "combine_ms": round(comb, 4),
                      "ingest_alg_bytes": ing_bytes, "ingest_alg_gbps": round(ing_bytes / (ing * 1e-3) / 1e9, 1),
                      "codes": {int(c): int(k) for c, k in zip(*np.unique(codes, return_counts=True))}}))
    fb.free()
    eng.close()


if __name__ == "__main__":
    main()
