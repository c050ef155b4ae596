"""Key cache (FDGPU_FLAG_KEY_CACHE) on its own: device-resident verifies of
cfg1-shaped batches whose signers come from pools of K keys (0 = a fresh key
per signer, cfg1 itself), with and without the cache; HIP-event timing.

    python tools/keycache_probe.py [--txns 1000000] [--pools 0,65536,4096,256]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from firedancer_amd import VerifyEngine, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=1_000_000)
    ap.add_argument("--pools", default="0,65536,4096,256")
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    plain = VerifyEngine(0, max_txn=1024, ring_depth=1)
    kc = VerifyEngine(0, max_txn=1024, ring_depth=1, key_cache=True)
    for pool in (int(p) for p in args.pools.split(",")):
        arena, txns, modes = workload.make_txns(args.txns, workload.CFG1_SEED + 0x600 + pool, key_pool=pool)
        row = {"txns": args.txns, "key_pool": pool}
        codes = {}
        for tag, e in (("plain", plain), ("kc", kc)):
            b = e.upload(arena, txns)
            b.verify()
            codes[tag] = b.codes()
            _, kv, kcomb = b.time(args.iters)
            row[f"{tag}_ms"] = round(kv + kcomb, 3)
            row[f"{tag}_sigs_per_s"] = round(b.n_sig / ((kv + kcomb) * 1e-3), 1)
            b.free()
        row["codes_equal"] = bool((codes["plain"] == codes["kc"]).all())
        row["self_check"] = bool(((codes["kc"] == 0) == (modes == 0)).all())
        row["speedup"] = round(row["plain_ms"] / row["kc_ms"], 3)
        print(json.dumps(row), flush=True)
    kc.close()
    plain.close()


if __name__ == "__main__":
    main()
