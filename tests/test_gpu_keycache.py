"""Key cache (FDGPU_FLAG_KEY_CACHE): each distinct public key of a batch is
decoded once and its -A table shared by the batch's other signatures of that
key.  The codes must not change, so every case here is held to the oracle
(and to the engine without the cache):

* the golden vectors (reference codes), AVX-512 and portable error mapping;
* signer pools of 1, 7, 64 and 4096 keys over cfg1/cfg3-shaped txns with the
  default corruption mix (bad signature / message / public key);
* the small-order x S-edge cross product (every A repeats 8 x |encodings|
  times, non-canonical and small-order keys included);
* the full-length fallback path (FDGPU_FLAG_FULL_PATH) reading copied tables;
* device batches (upload + re-verify) and GPU-parsed frag batches, where the
  signature count comes from the device.
"""
import numpy as np
import pytest

import firedancer_amd as fa
from firedancer_amd import workload

from test_gpu_parity import _vector_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kc_engine():
    e = fa.VerifyEngine(0, max_txn=1 << 15, max_sig=1 << 17, max_arena=1 << 26, key_cache=True)
    yield e
    e.close()


def test_key_cache_golden_vectors(kc_engine, vectors):
    vs, arena, txns = _vector_batch(vectors)
    codes = kc_engine.verify_txns(arena, txns)
    bad = [(v["src"], v["tc_id"], v["code"], int(c)) for v, c in zip(vs, codes) if c != v["code"]]
    assert not bad, bad[:20]


def test_key_cache_ref_mapping(vectors, oracle):
    eng = fa.VerifyEngine(0, max_txn=8192, ref_mapping=True, key_cache=True)
    try:
        vs, arena, txns = _vector_batch(vectors)
        codes = eng.verify_txns(arena, txns)
        bad = [(v["src"], v["tc_id"], v["code_refmap"], int(c)) for v, c in zip(vs, codes) if c != v["code_refmap"]]
        assert not bad, bad[:20]
        arena, txns = workload.pack_single(workload.small_order_cross_product())
        got = eng.verify_txns(arena, txns)
        assert (got == oracle.verify_txns(arena, txns, mapping=oracle.MAP_REF, nthreads=8)).all()
    finally:
        eng.close()


@pytest.mark.parametrize("pool,multi", [(1, False), (7, True), (64, False), (4096, False), (64, True)])
def test_key_pool_vs_oracle(kc_engine, engine, oracle, pool, multi):
    arena, txns, modes = workload.make_txns(6000 if not multi else 1500, 0x4B00 + pool, multi=multi, key_pool=pool)
    got = kc_engine.verify_txns(arena, txns)
    exp = oracle.verify_txns(arena, txns, nthreads=8)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    assert (engine.verify_txns(arena, txns) == got).all()
    assert (got == 0).sum() > 0.8 * len(txns) and (got != 0).sum() > 0.05 * len(txns)


def test_key_cache_cross_product(kc_engine, oracle):
    recs = workload.small_order_cross_product()
    arena, txns = workload.pack_single(recs)
    got = kc_engine.verify_txns(arena, txns)
    assert (got == oracle.verify_txns(arena, txns, nthreads=8)).all()


def test_key_cache_full_path(oracle):
    eng = fa.VerifyEngine(0, max_txn=8192, full_path=True, key_cache=True)
    try:
        arena, txns, _ = workload.make_txns(3000, 0x4B10, key_pool=16)
        got = eng.verify_txns(arena, txns)
        assert (got == oracle.verify_txns(arena, txns, nthreads=8)).all()
        arena, txns = workload.pack_single(workload.small_order_cross_product())
        assert (eng.verify_txns(arena, txns) == oracle.verify_txns(arena, txns, nthreads=8)).all()
    finally:
        eng.close()


def test_key_cache_device_and_frag_batches(kc_engine, engine, oracle):
    arena, txns, _ = workload.make_txns(20000, 0x4B20, key_pool=256)
    exp = oracle.verify_txns(arena, txns, nthreads=8)
    b = kc_engine.upload(arena, txns)
    for _ in range(2):                                   # re-verify: the hash table is cleared per launch
        b.verify()
        assert (b.codes() == exp).all()
    b.free()
    frags = np.zeros(len(txns), dtype=fa.ed25519.FRAG_DTYPE)
    frags["off"] = txns["sig_off"] - 1
    frags["sz"] = txns["msg_off"] + txns["msg_sz"] - frags["off"]
    pb = engine.upload_frags(arena, frags)
    pb.verify()
    plain = pb.codes()
    pb.free()
    fb = kc_engine.upload_frags(arena, frags)
    fb.verify()
    got = fb.codes()
    fb.free()
    # corrupted message bytes can make a payload unparsable (FDGPU_CODE_PARSE_FAIL)
    ok = plain != fa.ed25519.CODE_PARSE_FAIL
    assert (got == plain).all() and (got[ok] == exp[ok]).all() and ok.sum() > 0.99 * len(ok)
