"""Full-scale parity run (the north-star target):
>= 10M mixed valid/invalid signatures through the GPU engine, compared code
for code with the CPU oracle (oracle/, the C restatement pinned by the
reference's own vectors).  Run on the GPU box:

    python tools/parity_10m.py --out gpurun_out/parity10m.json

Parts (all compared per transaction, i.e. fd_ed25519_verify_batch_single_msg
codes, and the multi-signature part additionally per signature, i.e.
fd_ed25519_verify codes of every (R||S, A, msg) it contains):
  golden     every vector of tests/golden (cctv, wycheproof, malleability)
  cross      small-order / non-canonical A x R x S-edge cross product
  quic       the reference's 1000-txn QUIC corpus (src/waltz/quic/tests/txn/tx)
  cfg1       single-signature txns, 10% one-bit corrupted
  cfg3       1-12 signature txns sharing one message, msg <= 1232 B
--key-cache runs the engine with FDGPU_FLAG_KEY_CACHE and --key-pool K draws
the cfg1/cfg3 signers from K keys (signer reuse), so the key cache is held
to the same bar.
Exit status 1 on any mismatch.
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
from oracle import oracle as orc  # noqa: E402  (checker only)

T0 = time.time()


def log(*a):
    print(f"[{time.time() - T0:7.1f}s]", *a, flush=True)


def chunks(arena, txns, chunk):
    for i in range(0, len(txns), chunk):
        t = txns[i:i + chunk].copy()
        cnt = np.maximum(t["sig_cnt"].astype(np.int64), 1)
        lo = int(min(t["sig_off"].min(), t["msg_off"].min(), t["pub_off"].min()))
        hi = int(max((t["msg_off"].astype(np.int64) + t["msg_sz"]).max(),
                     (t["sig_off"].astype(np.int64) + 64 * cnt).max(),
                     (t["pub_off"].astype(np.int64) + 32 * cnt).max()))
        for f in ("msg_off", "sig_off", "pub_off"):
            t[f] -= lo
        yield i, np.ascontiguousarray(arena[lo:hi]), t


def gpu_codes(eng, arena, txns, chunk):
    out = np.empty(len(txns), dtype=np.int8)
    for i, a, t in chunks(arena, txns, chunk):
        out[i:i + len(t)] = eng.verify_txns(a, t)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg1", type=int, default=6_200_000, help="single-signature txns")
    ap.add_argument("--cfg3", type=int, default=600_000, help="multi-signature txns")
    ap.add_argument("--threads", type=int, default=workload.default_threads())
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "parity10m.json"))
    ap.add_argument("--key-cache", action="store_true", help="engine with FDGPU_FLAG_KEY_CACHE")
    ap.add_argument("--key-pool", type=int, default=0, help="cfg1/cfg3 signers from this many keys (0: fresh)")
    args = ap.parse_args()

    eng = fa.VerifyEngine(0, max_txn=1 << 17, max_sig=1 << 21, max_arena=1 << 28, key_cache=args.key_cache)
    parts = []

    def check(name, arena, txns, per_sig):
        t = time.time()
        got = gpu_codes(eng, arena, txns, 1 << 17)
        tg = time.time() - t
        t = time.time()
        exp = orc.verify_txns(arena, txns, nthreads=args.threads)
        tc = time.time() - t
        mism = int((got != exp).sum())
        rec = {"part": name, "txns": int(len(txns)), "sigs": int(np.clip(txns["sig_cnt"], 0, 16).sum()),
               "txn_mismatches": mism, "codes": {int(c): int(n) for c, n in zip(*np.unique(exp, return_counts=True))},
               "gpu_s": round(tg, 2), "oracle_s": round(tc, 2)}
        if mism:
            rec["first_mismatch"] = [int(i) for i in np.nonzero(got != exp)[0][:5]]
        if per_sig:
            st, _ = workload.explode_sigs(txns)
            sg = gpu_codes(eng, arena, st, 1 << 17)
            se = orc.verify_txns(arena, st, nthreads=args.threads)
            rec["per_sig_checked"] = int(len(st))
            rec["sig_mismatches"] = int((sg != se).sum())
            rec["sig_codes"] = {int(c): int(n) for c, n in zip(*np.unique(se, return_counts=True))}
        log(json.dumps(rec))
        parts.append(rec)

    vec = json.load(open(os.path.join(REPO, "tests", "golden", "ed25519_vectors.json")))["vectors"]
    recs = [(bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["pub"])) for v in vec]
    a, t = workload.pack_single(recs)
    check("golden", a, t, False)
    assert eng.verify_txns(a, t).tolist() == [v["code"] for v in vec], "golden codes differ from fixtures"

    a, t = workload.pack_single(workload.small_order_cross_product())
    check("cross", a, t, False)

    q = np.load(os.path.join(REPO, "tests", "golden", "quic_txns.npz"))
    check("quic", q["arena"], q["txns"], True)

    n1 = args.cfg1
    t = time.time()
    a, tx, modes = workload.make_txns(n1, workload.CFG1_SEED + 0x100, multi=False, key_pool=args.key_pool)
    log(f"generated cfg1 {n1} txns in {time.time() - t:.1f}s")
    check("cfg1", a, tx, False)
    del a, tx, modes

    n3 = args.cfg3
    t = time.time()
    a, tx, modes = workload.make_txns(n3, workload.CFG3_SEED + 0x100, multi=True, key_pool=args.key_pool)
    log(f"generated cfg3 {n3} txns ({int(tx['sig_cnt'].sum())} sigs) in {time.time() - t:.1f}s")
    check("cfg3", a, tx, True)
    del a, tx, modes
    eng.close()

    total_sigs = sum(p["sigs"] for p in parts)
    total_checks = sum(p["sigs"] if "per_sig_checked" not in p else p["per_sig_checked"] for p in parts)
    bad = sum(p["txn_mismatches"] + p.get("sig_mismatches", 0) for p in parts)
    summary = {"what": "cfg4 full-scale parity: GPU engine vs CPU oracle, code for code",
               "key_cache": bool(args.key_cache), "key_pool": args.key_pool,
               "signatures": total_sigs, "per_signature_codes_compared": total_checks,
               "transactions": sum(p["txns"] for p in parts), "mismatches": bad, "parts": parts,
               "wall_s": round(time.time() - T0, 1)}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(summary, f, indent=1)
    log(f"DONE signatures={total_sigs} mismatches={bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
