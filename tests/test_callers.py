"""The other callers of the verify API, batched:
replay's fd_executor_txn_verify over a block (fd_executor.c:1157-1185) and
the shred FEC-set root check (fd_fec_resolver.c:438).  Expected codes come
from the oracle called once per item, exactly as the reference callers call
fd_ed25519_verify_batch_single_msg / fd_ed25519_verify.  CPU tests run the
batching host code over the oracle as the verifier; the GPU tests over the
MI355X engine."""
import random

import numpy as np
import pytest

from firedancer_amd import tile, workload
import tile_model
from test_tile import _mixed_stream


def _replay_expected(oracle, payloads):
    exp = []
    for p in payloads:
        sz, raw = tile.txn_parse(p)
        if not sz:
            exp.append(tile.REPLAY_PARSE_FAIL)
            continue
        mo, ms, so, po, sc = tile_model.txn_descriptor(p, raw)
        txns = np.array([(mo, ms, so, po, sc)], dtype=tile.TXN_DTYPE)
        exp.append(int(oracle.verify_txns(np.frombuffer(p, dtype=np.uint8), txns)[0]))
    return exp


def _fec_sets(n, seed, shared=True):
    rnd = random.Random(seed)
    leader = bytes(rnd.randrange(256) for _ in range(32))
    roots, sigs, pubs, modes = [], [], [], []
    for i in range(n):
        prv = leader if shared else bytes(rnd.randrange(256) for _ in range(32))
        root = bytes(rnd.randrange(256) for _ in range(32))
        pub, sig = workload.sign(prv, root)
        mode = rnd.randrange(4) if rnd.random() < 0.2 else 0
        if mode == 1:                                          # forged root
            root = bytes([root[0] ^ 1]) + root[1:]
        elif mode == 2:                                        # bad signature bit
            b = rnd.randrange(512)
            sig = bytearray(sig); sig[b // 8] ^= 1 << (b % 8); sig = bytes(sig)
        elif mode == 3:                                        # S + L (non-canonical S)
            s = int.from_bytes(sig[32:], "little") + (2**252 + 27742317777372353535851937790883648493)
            if s < 2**256:
                sig = sig[:32] + s.to_bytes(32, "little")
        roots.append(root); sigs.append(sig); pubs.append(pub); modes.append(mode)
    pk = pubs[0] if shared else b"".join(pubs)
    return b"".join(roots), b"".join(sigs), pk, pubs, modes


def _fec_expected(oracle, roots, sigs, pubs):
    return [oracle.verify(roots[32 * i:32 * i + 32], sigs[64 * i:64 * i + 64], pubs[i]) for i in range(len(pubs))]


@pytest.mark.parametrize("batch_txn_max,slots", [(1, 1), (7, 2), (4096, 2)])
def test_replay_verify_vs_per_txn(oracle, quic_corpus, batch_txn_max, slots):
    """Every txn of a block gets exactly the code fd_executor_txn_verify's
    single call would see, for any batch cut (incl. the byte limit and a
    one-slot verifier that forces draining before each submit)."""
    arena, txns, _ = quic_corpus
    ps = workload.payloads(arena, txns[:200]) + _mixed_stream(300, seed=41)
    exp = _replay_expected(oracle, ps)
    ver = tile.PyVerifier(lambda a, t: oracle.verify_txns(a, t), slots=slots)
    got = tile.replay_verify(ver, ps, batch_txn_max=batch_txn_max, batch_bytes_max=5000)
    assert got.tolist() == exp
    assert exp.count(tile.REPLAY_PARSE_FAIL) > 5 and exp.count(0) > 200 and sum(e < 0 for e in exp) > 10


def test_replay_verify_empty_and_bad_args(oracle):
    ver = tile.PyVerifier(lambda a, t: oracle.verify_txns(a, t))
    assert len(tile.replay_verify(ver, [])) == 0
    with pytest.raises(RuntimeError):
        tile.replay_verify(ver, [b"x"], batch_bytes_max=100)         # below one MTU


@pytest.mark.parametrize("shared", [True, False])
def test_fec_roots_verify_vs_per_set(oracle, shared):
    roots, sigs, pk, pubs, modes = _fec_sets(300, seed=7 + shared, shared=shared)
    exp = _fec_expected(oracle, roots, sigs, pubs)
    ver = tile.PyVerifier(lambda a, t: oracle.verify_txns(a, t), slots=2)
    got = tile.fec_roots_verify(ver, roots, sigs, pk, batch_max=64)
    assert got.tolist() == exp
    assert exp.count(0) == modes.count(0) and exp.count(0) < len(exp)


@pytest.mark.gpu
def test_replay_and_fec_on_gpu(oracle, quic_corpus, engine):
    arena, txns, _ = quic_corpus
    ps = workload.payloads(arena, txns) + _mixed_stream(2000, seed=43)
    ver = tile.EngineVerifier([engine])
    try:
        got = tile.replay_verify(ver, ps, batch_txn_max=1024, batch_bytes_max=1024 * 1232)
        assert got.tolist() == _replay_expected(oracle, ps)
        roots, sigs, pk, pubs, _ = _fec_sets(3000, seed=11, shared=True)
        got = tile.fec_roots_verify(ver, roots, sigs, pk, batch_max=1024)
        assert got.tolist() == _fec_expected(oracle, roots, sigs, pubs)
    finally:
        ver.close()
