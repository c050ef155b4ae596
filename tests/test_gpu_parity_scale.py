"""North-star parity on the GPU (BASELINE configs[3] / SURVEY §8(d) cfg4):

* the reference's fuzz corpus (corpus/fuzz_ed25519_sigverify, harness
  fuzz_ed25519_sigverify.c:23-50: prv||msg -> sign -> verify must succeed)
  through the engine, plus every single-bit neighbour of each record's
  (sig, pub, msg) -- the harness's input space one flip away -- code for code
  against the oracle, and the fuzz_ed25519_verify.c:31-48 property (random
  sig||pub||msg must fail);
* >= 10M mixed valid / invalid signatures through the engine, every
  transaction code (and a sample of per-signature codes) compared with the
  oracle: the golden vectors, the small-order cross product, the QUIC
  corpus, 4M cfg1 single-signature txns (fresh keys, the bench workload's
  generator) and 1M cfg3 multi-signature txns (~6.5M signatures, signers
  from a key pool, messages up to the 1232-B MTU).
"""
import os
import sys
import time

import numpy as np
import pytest

from firedancer_amd import workload

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))


def _log(*a):
    print(f"[parity {time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


def _chunks(arena, txns, chunk):
    """(start, arena slice, rebased txns) per chunk of txns (contiguous records)."""
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


def _compact(arena, txns):
    """The records txns point at, copied back to back into a fresh arena
    (signatures, public keys, message per txn) with rebased descriptors."""
    parts, out, off = [], txns.copy(), 0
    for i, t in enumerate(txns):
        cnt = int(t["sig_cnt"]) if 1 <= int(t["sig_cnt"]) <= 16 else 1
        for f, n in (("sig_off", 64 * cnt), ("pub_off", 32 * cnt), ("msg_off", int(t["msg_sz"]))):
            parts.append(arena[int(t[f]):int(t[f]) + n])
            out[i][f] = off
            off += n
    return np.concatenate(parts) if parts else np.zeros(1, np.uint8), out


def _gpu_codes(eng, arena, txns, chunk=1 << 17):
    out = np.empty(len(txns), dtype=np.int8)
    for i, a, t in _chunks(arena, txns, chunk):
        out[i:i + len(t)] = eng.verify_txns(a, t)
    return out


@pytest.fixture(scope="module")
def big_engine():
    from firedancer_amd import VerifyEngine
    e = VerifyEngine(0, max_txn=1 << 17, max_arena=1 << 28)       # max_sig: 12 per txn
    yield e
    e.close()


def _flip(b, bit):
    b = bytearray(b)
    b[bit // 8] ^= 1 << (bit % 8)
    return bytes(b)


def test_fuzz_corpus_on_gpu(big_engine, misc_vectors, oracle):
    import firedancer_amd as fa
    recs = misc_vectors["fuzz"]
    assert len(recs) == 4
    base = []
    for f in recs:
        msg, sig, pub = bytes.fromhex(f["msg"]), bytes.fromhex(f["sig"]), bytes.fromhex(f["pub"])
        base.append((msg, sig, pub))
        assert fa.verify(msg, sig, pub) == fa.SUCCESS                # the harness's assert, sync API
    a, t = workload.pack_single(base)
    assert big_engine.verify_txns(a, t).tolist() == [0] * 4      # batch API
    # every single-bit neighbour of every record (sig: 512, pub: 256, msg: 8 x len)
    neigh = []
    for msg, sig, pub in base:
        neigh += [(msg, _flip(sig, b), pub) for b in range(512)]
        neigh += [(msg, sig, _flip(pub, b)) for b in range(256)]
        neigh += [(_flip(msg, b), sig, pub) for b in range(8 * len(msg))]
    a, t = workload.pack_single(neigh)
    got = big_engine.verify_txns(a, t)
    exp = oracle.verify_txns(a, t)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    assert set(np.unique(exp).tolist()) <= {0, -1, -2, -3} and (exp != 0).sum() > 0.9 * len(exp)
    # fuzz_ed25519_verify.c:31-48: random sig || pub || msg must not verify
    rng = np.random.default_rng(0xF022)
    rnd = [(rng.bytes(int(rng.integers(0, 300))), rng.bytes(64), rng.bytes(32)) for _ in range(4096)]
    a, t = workload.pack_single(rnd)
    got = big_engine.verify_txns(a, t)
    assert (got == oracle.verify_txns(a, t)).all() and (got != 0).all()


def test_parity_10m(big_engine, vectors, oracle, quic_corpus):
    """>= 10M signatures, every transaction code vs the oracle (this is the
    north-star target run as a driver-observed test)."""
    eng, cpus = big_engine, workload.physical_cpus()
    total_sigs, mism = 0, 0
    t0 = time.time()

    def check(name, arena, txns, per_sig_sample=0):
        nonlocal total_sigs, mism
        got = _gpu_codes(eng, arena, txns)
        exp = oracle.verify_txns(arena, txns, cpus=cpus)
        bad = int((got != exp).sum())
        n_sig = int(np.where((txns["sig_cnt"] >= 1) & (txns["sig_cnt"] <= 16), txns["sig_cnt"], 0).sum())
        msg = f"{name}: {len(txns)} txns / {n_sig} sigs, {bad} mismatches, codes " \
              f"{dict(zip(*[x.tolist() for x in np.unique(exp, return_counts=True)]))}"
        if per_sig_sample:
            idx = np.sort(np.random.default_rng(7).choice(len(txns), min(per_sig_sample, len(txns)), replace=False))
            ca, ct = _compact(arena, txns[idx])
            st, _ = workload.explode_sigs(ct)
            sg = _gpu_codes(eng, ca, st)
            se = oracle.verify_txns(ca, st, cpus=cpus)
            bad += int((sg != se).sum())
            msg += f"; per-signature sample {len(st)}: {int((sg != se).sum())} mismatches"
        _log(msg, f"({time.time() - t0:.0f}s)")
        total_sigs += n_sig
        mism += bad

    recs = [(bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["pub"])) for v in vectors["vectors"]]
    a, t = workload.pack_single(recs)
    check("golden", a, t)
    a, t = workload.pack_single(workload.small_order_cross_product())
    check("cross", a, t)
    check("quic", quic_corpus[0], quic_corpus[1], per_sig_sample=1000)
    n1 = 4_000_000
    a, t, _ = workload.make_txns(n1, workload.CFG1_SEED + 0x100)
    check("cfg1", a, t)
    del a, t
    n3 = 1_000_000
    a, t, _ = workload.make_txns(n3, workload.CFG3_SEED + 0x100, multi=True, key_pool=1 << 16)
    check("cfg3", a, t, per_sig_sample=50_000)
    del a, t
    _log(f"total {total_sigs} signatures, {mism} mismatches, {time.time() - t0:.0f}s")
    assert total_sigs >= 10_000_000
    assert mism == 0
