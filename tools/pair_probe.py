"""One lane vs two lanes per signature (FDGPU_FLAG_PAIR) on device-resident
cfg1 batches of several sizes: the verify kernel's mean duration by HIP
events (fdgpu_dev_batch_time), codes compared between the two kernels.  The
pair kernel halves a wave's dependent chain of field products per signature
(one decompression and a one-table chain per lane) at ~1.4x the work, so it
wins while a batch leaves wave slots idle and loses once the GPU is full.

    python tools/pair_probe.py [--sizes 1,64,4096,16384,65536,262144,1048576] [--out f.jsonl]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import firedancer_amd as fa  # noqa: E402
from firedancer_amd import workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,64,2048,4096,8192,16384,32768,65536,131072,262144,1048576")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    sizes = [int(x) for x in args.sizes.split(",")]
    arena, txns, _ = workload.cfg1(max(sizes), seed=0x9A12)
    engs = {p: fa.VerifyEngine(0, max_txn=max(sizes), max_sig=2 * max(sizes), max_arena=max(sizes) * 400, pair=p)
            for p in (False, True)}
    lines = []
    for n in sizes:
        t = txns[:n]
        res = {"sigs": n}
        codes = {}
        for p, e in engs.items():
            b = e.upload(arena, t)
            b.verify()
            codes[p] = b.codes()
            wall, kv, kc = b.time(args.iters)
            res["pair" if p else "one"] = {"verify_kernel_ms": round(kv, 4), "wall_ms": round(wall, 4)}
            b.free()
        res["codes_equal"] = bool((codes[False] == codes[True]).all())
        res["pair_vs_one"] = round(res["pair"]["verify_kernel_ms"] / res["one"]["verify_kernel_ms"], 3)
        print(json.dumps(res), flush=True)
        lines.append(json.dumps(res))
    for e in engs.values():
        e.close()
    if args.out:
        with open(args.out, "w") as f:
            f.write("\n".join(lines) + "\n")
    return 0 if all(json.loads(x)["codes_equal"] for x in lines) else 1


if __name__ == "__main__":
    sys.exit(main())
