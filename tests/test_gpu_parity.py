"""GPU parity: every stage of the MI355X path against the CPU oracle / exact
integer arithmetic, and whole-path result codes against the golden vectors.
Bit-exact everywhere (integer/byte work; no tolerance applies)."""
import hashlib
import random

import numpy as np
import pytest

import pyref_ed25519 as pyref
from firedancer_amd import workload
import firedancer_amd as fa

pytestmark = pytest.mark.gpu

P, L = pyref.P, pyref.L


def _le(x, n=32):
    return int(x % (1 << (8 * n))).to_bytes(n, "little")


# ------------------------------------------------------------ field layer

def test_field_ops(engine):
    rnd = random.Random(11)
    edge = [0, 1, 2, 19, P - 1, P, P + 1, P + 18, 2**255 - 1, 2**255 - 20, 2**254, 2**26 - 1, 2**51 + 7]
    vals = edge + [rnd.getrandbits(255) for _ in range(500)]
    pairs = [(a, b) for a in edge for b in edge] + [(rnd.choice(vals), rnd.choice(vals)) for _ in range(1500)]
    ab = np.frombuffer(b"".join(_le(a) + _le(b) for a, b in pairs), dtype=np.uint8)
    out = engine.debug_fe_ops(ab)
    for i, (a, b) in enumerate(pairs):
        a %= 2**255; b %= 2**255
        got = [int.from_bytes(out[i, k].tobytes(), "little") for k in range(8)]
        exp = [a * b % P, a * a % P, (a + b) % P, (a - b) % P, pow(a, (P - 5) // 8, P),
               pow(a, P - 2, P), a % P, (-a) % P]
        assert got == exp, (i, hex(a), hex(b), [g == e for g, e in zip(got, exp)])


def test_scalar_reduce(engine):
    rnd = random.Random(5)
    xs = [0, 1, L - 1, L, L + 1, 2**512 - 1, L * L, (L - 1) * 2**259, 2**511] + [rnd.getrandbits(512) for _ in range(2000)]
    xs = [x % 2**512 for x in xs]
    out = engine.debug_sc_reduce(np.frombuffer(b"".join(_le(x, 64) for x in xs), dtype=np.uint8))
    for i, x in enumerate(xs):
        assert int.from_bytes(out[i].tobytes(), "little") == x % L, i


# ------------------------------------------------------------ SHA-512

def _msgs_arena(msgs, misalign=0):
    chunks, txns, off = [], [], misalign
    for m in msgs:
        chunks.append(m)
        txns.append((off, len(m), 0, 0, 1))
        off += len(m)
    arena = np.frombuffer(b"\0" * misalign + b"".join(chunks) + b"\0", dtype=np.uint8)
    return arena, np.array(txns, dtype=fa.TXN_DTYPE)


def test_sha512_cavp(engine, sha_vectors):
    msgs = [bytes.fromhex(v["msg"]) for v in sha_vectors["short"] + sha_vectors["long"]]
    for mis in (0, 1, 3):
        arena, txns = _msgs_arena(msgs, mis)
        out = engine.debug_sha512(arena, txns)
        for i, v in enumerate(sha_vectors["short"] + sha_vectors["long"]):
            assert out[i].tobytes().hex() == v["md"], (mis, i, len(msgs[i]))


def test_sha512_all_lengths(engine):
    rnd = random.Random(9)
    msgs = [rnd.randbytes(n) for n in range(0, 1300)]
    rnd.shuffle(msgs)                       # mixed block counts inside each wave
    arena, txns = _msgs_arena(msgs, 2)
    out = engine.debug_sha512(arena, txns)
    for i, m in enumerate(msgs):
        assert out[i].tobytes() == hashlib.sha512(m).digest(), len(m)


def test_hram_mod_l(engine):
    """k = SHA-512(R || A || M) mod L (fd_ed25519_user.c:205-207), all message
    lengths around the block boundaries, unaligned offsets."""
    rnd = random.Random(4)
    recs, chunks, txns, off = [], [], [], 1
    for n in list(range(0, 300)) + [1232 - 65, 1100, 1167]:
        R, A, M = rnd.randbytes(32), rnd.randbytes(32), rnd.randbytes(n)
        chunks += [R + rnd.randbytes(32), A, M]
        txns.append((off + 96, n, off, off + 64, 1))
        off += 96 + n
        recs.append((R, A, M))
    arena = np.frombuffer(b"\0" + b"".join(chunks), dtype=np.uint8)
    out = engine.debug_hram(arena, np.array(txns, dtype=fa.TXN_DTYPE))
    for i, (R, A, M) in enumerate(recs):
        k = int.from_bytes(hashlib.sha512(R + A + M).digest(), "little") % L
        assert int.from_bytes(out[i].tobytes(), "little") == k, i


# ------------------------------------------------------------ point decoding

def _special_encodings():
    enc = []
    ys = [0, 1, 2, P - 1, P - 2, P, P + 1, P + 2, P + 18, 2**255 - 1, 2**255 - 19, 2**255 - 20, 19, 20]
    y0 = int("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05", 16)
    for y in ys:
        for s in (0, 1):
            enc.append(_le(y + (s << 255)))
    for h in ["26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05",
              "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a",
              "5866666666666666666666666666666666666666666666666666666666666666",
              "b898e00f6f6df758b3f9a05cbf73b15fd392a008a9a417d471c178c1b28c7447"]:
        b = bytes.fromhex(h)
        enc += [b, b[:31] + bytes([b[31] ^ 0x80])]
    del y0
    return enc


def test_decode_and_small_order(engine, oracle, vectors):
    rnd = random.Random(8)
    enc = _special_encodings()
    for v in vectors["vectors"]:
        enc += [bytes.fromhex(v["pub"]), bytes.fromhex(v["sig"])[:32]]
    enc += [rnd.randbytes(32) for _ in range(1000)]
    arr = np.frombuffer(b"".join(enc), dtype=np.uint8)
    for mapping, refm in ((oracle.MAP_AVX512, False), (oracle.MAP_REF, True)):
        rc, so, x, y = engine.debug_decode(arr, ref_mapping=refm)
        for i, e in enumerate(enc):
            orc_rc, orc_so, xy = oracle.point_decode(e, mapping)
            assert rc[i] == orc_rc, (mapping, e.hex())
            if orc_rc == 0:
                assert so[i] == orc_so, (mapping, e.hex())
                assert x[i].tobytes() == xy[:32] and y[i].tobytes() == xy[32:], (mapping, e.hex())


# ------------------------------------------------------------ whole path

def _vector_batch(vectors, src=None):
    vs = [v for v in vectors["vectors"] if src is None or v["src"] == src]
    arena, txns = workload.pack_single((bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["pub"]))
                                       for v in vs)
    return vs, arena, txns


def test_golden_vectors_avx512_codes(engine, vectors):
    vs, arena, txns = _vector_batch(vectors)
    codes = engine.verify_txns(arena, txns)
    bad = [(v["src"], v["tc_id"], v["code"], int(c)) for v, c in zip(vs, codes) if c != v["code"]]
    assert not bad, bad[:20]
    sig_codes = engine.debug_sig_codes(arena, txns)
    assert (sig_codes == codes).all()


def test_golden_vectors_ref_mapping(engine_ref, vectors):
    vs, arena, txns = _vector_batch(vectors)
    codes = engine_ref.verify_txns(arena, txns)
    bad = [(v["src"], v["tc_id"], v["code_refmap"], int(c)) for v, c in zip(vs, codes) if c != v["code_refmap"]]
    assert not bad, bad[:20]


def test_cctv_batch(engine, vectors):
    b = vectors["cctv_batch"]
    msg, sigs, pubs = (bytes.fromhex(b[k]) for k in ("msg", "sigs", "pubs"))
    cctv = [v for v in vectors["vectors"] if v["src"] == "cctv"]
    chunks, txns, exp, off = [], [], [], 0
    for case in b["cases"]:
        v = cctv[case["cctv_index"]]
        s = bytearray(sigs); p = bytearray(pubs)
        s[64:128] = bytes.fromhex(v["sig"]); p[32:64] = bytes.fromhex(v["pub"])
        for n, code in ((2, case["code2"]), (4, case["code4"])):
            chunks += [bytes(s[:64 * n]), bytes(p[:32 * n]), msg]
            txns.append((off + 96 * n, len(msg), off, off + 64 * n, n))
            off += 96 * n + len(msg)
            exp.append(code)
    chunks += [sigs, pubs, msg]
    txns.append((off + 96 * 16, len(msg), off, off + 64 * 16, 16)); exp.append(0)
    arena = np.frombuffer(b"".join(chunks), dtype=np.uint8)
    codes = engine.verify_txns(arena, np.array(txns, dtype=fa.TXN_DTYPE))
    assert codes.tolist() == exp


def test_txn_fixtures(engine, txn_fixtures):
    chunks, txns, off = [], [], 0
    for t in txn_fixtures:
        p = bytes.fromhex(t["payload"])
        chunks.append(p)
        txns.append((off + t["msg_off"], len(p) - t["msg_off"], off + t["sig_off"], off + t["pub_off"], t["sig_cnt"]))
        off += len(p)
    arena = np.frombuffer(b"".join(chunks), dtype=np.uint8)
    codes = engine.verify_txns(arena, np.array(txns, dtype=fa.TXN_DTYPE))
    assert codes.tolist() == [t["code"] for t in txn_fixtures]
    sig_codes = engine.debug_sig_codes(arena, np.array(txns, dtype=fa.TXN_DTYPE))
    assert sig_codes.tolist() == [c for t in txn_fixtures for c in t["sig_codes"]]


def test_quic_corpus(engine, quic_corpus):
    arena, txns, codes = quic_corpus
    assert (engine.verify_txns(arena, txns) == codes).all()


def test_cfg1_random_vs_oracle(engine, oracle):
    arena, txns, modes = workload.cfg1(3000, seed=0x1234)
    got = engine.verify_txns(arena, txns)
    exp = oracle.verify_txns(arena, txns, nthreads=8)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    assert (got[modes == 0] == 0).all() and (got[modes != 0] != 0).all()


def test_cfg3_multisig_vs_oracle(engine, oracle):
    arena, txns, modes = workload.cfg3(1500, seed=0x4321)
    got = engine.verify_txns(arena, txns)
    exp = oracle.verify_txns(arena, txns, nthreads=8)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]


def test_small_order_cross_product(engine, oracle):
    """small-order encodings (and y+p variants, sign bits) as
    A x R with S in {0, 1, L-1, L, L+1, 2^253-1, 2^256-1}."""
    recs = workload.small_order_cross_product()
    arena, txns = workload.pack_single(recs)
    got = engine.verify_txns(arena, txns)
    exp = oracle.verify_txns(arena, txns, nthreads=8)
    assert len(recs) > 1000
    assert (got == exp).all(), [recs[i] for i in np.nonzero(got != exp)[0][:3]]


def test_batch_edges(engine, oracle):
    """sig_cnt 0 and 17 -> ERR_SIG; empty and maximal messages; empty batch."""
    prv = bytes(range(1, 33))
    recs = []
    for n in (0, 1, 127, 128, 129, 1232 - 65):
        msg = bytes((i * 7) & 255 for i in range(n))
        pub, sig = workload.sign(prv, msg)
        recs.append((msg, sig, pub))
    arena, txns = workload.pack_single(recs)
    txns = np.concatenate([txns, txns[:2].copy(), txns[:1].copy()])
    txns["sig_cnt"][-3] = 0
    txns["sig_cnt"][-2] = 17
    txns["sig_cnt"][-1] = 1
    codes = engine.verify_txns(arena, txns)
    assert codes.tolist() == [0] * 6 + [-1, -1, 0]
    assert engine.verify_txns(arena, txns[:0]).tolist() == []


def test_sync_api(vectors):
    """fd_ed25519_verify / fd_ed25519_verify_batch_single_msg through the C ABI."""
    vs = vectors["vectors"][:40] + vectors["vectors"][-10:]
    for v in vs:
        msg, sig, pub = (bytes.fromhex(v[k]) for k in ("msg", "sig", "pub"))
        assert fa.verify(msg, sig, pub) == v["code"]
    prv = bytes(range(32))
    pub, sig = workload.sign(prv, b"batch")
    assert fa.verify_batch_single_msg(b"batch", sig * 3, pub * 3, None, 3) == 0
    assert fa.verify_batch_single_msg(b"batch", sig, pub, None, 0) == -1
    assert fa.verify_batch_single_msg(b"batch", sig * 17, pub * 17, None, 17) == -1


def test_async_ring(engine):
    a1, t1, m1 = workload.cfg1(700, seed=1)
    a2, t2, m2 = workload.cfg1(900, seed=2)
    k1 = engine.submit(a1, t1)
    k2 = engine.submit(a2, t2)
    with pytest.raises(RuntimeError):
        engine.submit(a1, t1)               # both slots hold unpolled batches
    c2 = engine.poll(k2, blocking=True)
    c1 = engine.poll(k1, blocking=True)
    assert ((c1 == 0) == (m1 == 0)).all() and ((c2 == 0) == (m2 == 0)).all()
    k3 = engine.submit(a1, t1)
    while True:
        c3 = engine.poll(k3, blocking=False)
        if c3 is not None:
            break
    assert (c3 == c1).all()


def test_threaded_staging_large_arena(engine, oracle):
    """Arenas >= 4 MB are staged by 4 host threads, each queuing its part's
    upload (fdgpu_engine.cpp stage_arena); sizes straddle the part rounding."""
    arena, txns, _ = workload.cfg1(24000, seed=0x5151)
    exp = oracle.verify_txns(arena, txns, nthreads=8)
    dev = engine.upload(arena, txns)
    dev.verify()
    assert (dev.codes() == exp).all()
    for n in (13000, 13001, 24000):          # 4.3 MB .. 7.9 MB arenas
        t = txns[:n]
        hi = int((t["msg_off"] + t["msg_sz"]).max())
        assert hi >= 4 << 20
        got = engine.verify_txns(np.ascontiguousarray(arena[:hi]), t)
        assert (got == exp[:n]).all(), (n, np.nonzero(got != exp[:n])[0][:10])


def test_device_resident_batch(engine):
    """Batch staged in HBM once, verified repeatedly (the benchmark path)."""
    arena, txns, modes = workload.cfg3(3000, seed=77)
    b = engine.upload(arena, txns)
    assert b.n_sig == int(txns["sig_cnt"].sum())
    b.verify()
    t1, s1 = b.codes(sig_codes=True)
    b.verify(); b.verify()
    t2 = b.codes()
    assert (t1 == t2).all()
    assert (t1 == engine.verify_txns(arena, txns)).all()
    assert (s1 == engine.debug_sig_codes(arena, txns)).all()
    wall, kv, kc = b.time(3)
    assert wall > 0 and 0 < kv <= wall and kc >= 0
    b.free()


def test_device_batches_own_queues(engine, oracle):
    """Batches on their own streams + workspaces (the bench's overlapped
    steps): concurrent verifies of different batches and of the compute-stream
    path give the oracle's codes, and engine.sync() covers every queue."""
    sets = [workload.cfg1(70000, seed=0x0A01), workload.cfg3(4000, seed=0x0A02), workload.cfg1(3001, seed=0x0A03)]
    exp = [oracle.verify_txns(a, t, nthreads=8) for a, t, _ in sets]
    bs = [engine.upload(a, t).own_queue() for a, t, _ in sets]
    shared = engine.upload(*sets[2][:2])                 # engine compute stream, engine workspace
    for _ in range(3):
        for b in bs:
            b.verify()
        shared.verify()
    engine.sync()
    for b, e in zip(bs, exp):
        assert (b.codes() == e).all()
    assert (shared.codes() == exp[2]).all()
    wall, kv, kc = bs[0].time(2)
    assert wall > 0 and 0 < kv <= wall
    for b in bs + [shared]:
        b.free()


def test_raw_device_pointer_api():
    """fdgpu_verify_device with device buffers the caller owns (here: an
    engine-owned DeviceBatch's, via fdgpu_dev_batch_device_ptrs; no torch
    involvement).  Descriptors in transaction order (FDGPU_FLAG_NO_BUCKET)."""
    import ctypes
    import firedancer_amd as fa
    from firedancer_amd import _lib
    arena, txns, modes = workload.cfg1(2000, seed=78)
    eng = fa.VerifyEngine(0, max_txn=4096, bucket=False)
    try:
        b = eng.upload(arena, txns)
        p = [ctypes.c_void_p() for _ in range(6)]
        assert _lib.lib().fdgpu_dev_batch_device_ptrs(b._b, *[ctypes.byref(x) for x in p]) == 0
        d_arena, d_sigs, d_perm, d_txns, d_sc, d_tc = [x.value for x in p]
        assert d_perm is None
        eng.verify_device(d_arena, d_sigs, b.n_sig, d_txns, b.n_txn, d_sc, d_tc, 0)
        eng.sync()
        assert ((b.codes() == 0) == (modes == 0)).all()
        b.free()
    finally:
        eng.close()


def test_full_size_cfg1_properties(engine, oracle):
    """BASELINE cfg2 at full size (1M txns): every untouched transaction
    verifies, every corrupted one fails, and a random 3000-txn sample matches
    the oracle code for code."""
    n = 1_000_000
    arena, txns, modes = workload.cfg1(n)
    codes = engine.verify_txns(arena, txns) if n <= engine._cfg.max_txn else _chunked(engine, arena, txns)
    assert (codes[modes == 0] == 0).all()
    assert (codes[modes != 0] != 0).all()
    idx = np.random.default_rng(1).choice(n, 3000, replace=False)
    exp = oracle.verify_txns(arena, txns[idx], nthreads=8)
    assert (codes[idx] == exp).all()


def _chunked(engine, arena, txns, chunk=1 << 17):
    out = []
    for i in range(0, len(txns), chunk):
        t = txns[i:i + chunk].copy()
        lo = int(t["sig_off"].min())
        hi = int((t["msg_off"] + t["msg_sz"]).max())
        for f in ("msg_off", "sig_off", "pub_off"):
            t[f] -= lo
        out.append(engine.verify_txns(arena[lo:hi], t))
    return np.concatenate(out)


def test_r_sign_and_equation_edges(engine, oracle):
    """Edges of the final equation check (chain == -[w]B, projective;
    fdgpu_verify_hs_kernel): R's sign bit flipped on
    valid signatures (decoded R = -R': ERR_MSG), R replaced by A or by B's
    encoding, S + L (out of range), and every lane of a batch failing the
    equation (settled in the one pass like every other lane)."""
    arena, txns, modes = workload.cfg1(2000, seed=0x5157)
    recs = []
    for t in txns[modes == 0][:600]:
        msg = bytes(arena[int(t["msg_off"]): int(t["msg_off"]) + int(t["msg_sz"])])
        sig = bytearray(arena[int(t["sig_off"]): int(t["sig_off"]) + 64])
        pub = bytes(arena[int(t["pub_off"]): int(t["pub_off"]) + 32])
        flipped = bytearray(sig); flipped[31] ^= 0x80
        recs.append((msg, bytes(flipped), pub))                        # R -> -R
        recs.append((msg, pub + bytes(sig[32:]), pub))                 # R = A
        s_plus_l = (int.from_bytes(sig[32:], "little") + L) % 2**256
        recs.append((msg, bytes(sig[:32]) + _le(s_plus_l), pub))       # S >= L
        recs.append((msg, bytes(sig), pub))                            # untouched
    a2, t2 = workload.pack_single(recs)
    got = engine.verify_txns(a2, t2)
    exp = oracle.verify_txns(a2, t2, nthreads=8)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    assert (exp[0::4] == -3).sum() > 590 and (exp[3::4] == 0).all()
    bad = np.nonzero(exp != 0)[0]                                      # an all-failing batch
    sub = t2[bad]
    got_bad = engine.verify_txns(a2, sub)
    assert (got_bad == exp[bad]).all()


def test_zero_copy_staging(engine):
    """fdgpu_stage_acquire / stage_submit / poll_keep / release: payloads
    written straight into the pinned slot verify like fdgpu_submit, the slot
    stays reserved until released, one staged slot at a time."""
    import ctypes
    L = fa._lib.lib() if hasattr(fa, "_lib") else __import__("firedancer_amd._lib", fromlist=["lib"]).lib()
    arena, txns, modes = workload.cfg1(500, seed=91)
    cap = ctypes.c_uint64()
    p = L.fdgpu_stage_acquire(engine._h, ctypes.byref(cap))
    assert p and cap.value >= len(arena)
    assert not L.fdgpu_stage_acquire(engine._h, ctypes.byref(cap))      # one staged slot per engine
    ctypes.memmove(p, arena.ctypes.data, len(arena))
    t = np.ascontiguousarray(txns)
    tk = L.fdgpu_stage_submit(engine._h, len(arena), t.ctypes.data, len(t))
    assert tk >= 0
    codes = np.zeros(len(t), dtype=np.int8)
    assert L.fdgpu_poll_keep(engine._h, tk, codes.ctypes.data, 1) == 0
    assert ((codes == 0) == (modes == 0)).all()
    assert bytes((ctypes.c_uint8 * 64).from_address(p)) == bytes(arena[:64])   # still reserved, intact
    assert (engine.verify_txns(arena, txns) == codes).all()
    assert L.fdgpu_release(engine._h, tk) == 0
    assert L.fdgpu_release(engine._h, tk) != 0
    p2 = L.fdgpu_stage_acquire(engine._h, ctypes.byref(cap))
    assert p2 and L.fdgpu_stage_cancel(engine._h) == 0


def test_block_count_grouping_keeps_codes(engine, oracle):
    """Signatures are verified grouped by SHA-512 block count (engine
    default) yet every code lands in the caller's order: transaction and
    per-signature codes equal the ungrouped engine's and the oracle's, over
    messages of 0 to 1100+ bytes (1 to 10 blocks) interleaved at random."""
    import firedancer_amd as fa
    a3, t3, _ = workload.cfg3(1200, seed=0xB0C)
    a1, t1, _ = workload.make_txns(1200, 0xB0D, msg_lo=0, msg_hi=1100)
    a1 = a1.copy()
    off = len(a3)
    t1 = t1.copy()
    for f in ("msg_off", "sig_off", "pub_off"):
        t1[f] += off
    arena = np.concatenate([a3, a1])
    txns = np.concatenate([t3, t1])[np.random.default_rng(5).permutation(len(t3) + len(t1))]
    flat = fa.VerifyEngine(0, max_txn=1 << 13, bucket=False)
    try:
        got, got_flat = engine.verify_txns(arena, txns), flat.verify_txns(arena, txns)
        sig, sig_flat = engine.debug_sig_codes(arena, txns), flat.debug_sig_codes(arena, txns)
        b = engine.upload(arena, txns)
        b.verify()
        dev_t, dev_s = b.codes(sig_codes=True)
        b.free()
    finally:
        flat.close()
    exp = oracle.verify_txns(arena, txns, nthreads=8)
    st, _ = workload.explode_sigs(txns)
    exp_s = oracle.verify_txns(arena, st, nthreads=8)
    assert (got == exp).all() and (got_flat == exp).all() and (dev_t == exp).all()
    assert (sig == exp_s).all() and (sig_flat == exp_s).all() and (dev_s == exp_s).all()


@pytest.mark.parametrize("mode", [workload.MODE_MSG, workload.MODE_R])
def test_all_failing_batches(engine, oracle, mode):
    """test_ed25519.c:920-951 bad-msg / bad-sig modes at batch scale: every
    signature of a 65,536-txn batch fails (the equation, or R's decode,
    across the whole grid -- the half-size kernel settles both in its one
    pass); codes vs the oracle."""
    arena, txns, modes = workload.make_txns(65536, 0xAD0 + mode, corrupt=1.0, corrupt_mode=mode)
    assert (modes == mode).all()
    got = engine.verify_txns(arena, txns)
    exp = oracle.verify_txns(arena, txns, nthreads=8)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    assert (got != 0).all()


def test_full_length_fallback_path(vectors, oracle):
    """The half-size kernel hands a lane whose lattice split fails (a Euclid
    quotient >= 2^31: ~2^-30 per step, no input reaches it on purpose) to
    fdgpu_full_kernel, the full-length [S]B + [k](-A) chain.  FDGPU_FLAG_FULL_PATH
    sends every signature there, so that path is held to the same parity bar:
    the golden vectors (reference codes), random cfg1/cfg3 sets and the
    small-order x S-edge cross product against the oracle."""
    import firedancer_amd as fa
    eng = fa.VerifyEngine(0, max_txn=8192, full_path=True)
    try:
        vs, arena, txns = _vector_batch(vectors)
        codes = eng.verify_txns(arena, txns)
        bad = [(v["src"], v["tc_id"], v["code"], int(c)) for v, c in zip(vs, codes) if c != v["code"]]
        assert not bad, bad[:20]
        for arena, txns, _ in (workload.cfg1(2000, seed=0xF011), workload.cfg3(600, seed=0xF012)):
            got = eng.verify_txns(arena, txns)
            exp = oracle.verify_txns(arena, txns, nthreads=8)
            assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
        arena, txns = workload.pack_single(workload.small_order_cross_product())
        got = eng.verify_txns(arena, txns)
        assert (got == oracle.verify_txns(arena, txns, nthreads=8)).all()
    finally:
        eng.close()


def test_engines_share_device_table(oracle):
    """Engines opened on one device share its fixed-base comb table
    (refcounted): closing the engine that built it leaves the others
    verifying correctly, a later open reuses the table, and concurrent
    batches of two engines give the oracle's codes."""
    arena, txns, _ = workload.cfg1(5000, seed=0x0B01)
    exp = oracle.verify_txns(arena, txns, nthreads=8)
    e1 = fa.VerifyEngine(0, max_txn=8192, ring_depth=2)
    e2 = fa.VerifyEngine(0, max_txn=8192, ring_depth=2)
    try:
        t1, t2 = e1.submit(arena, txns), e2.submit(arena, txns)
        assert (e1.poll(t1, blocking=True) == exp).all()
        assert (e2.poll(t2, blocking=True) == exp).all()
        e1.close()                                       # the table's builder goes first
        assert (e2.verify_txns(arena, txns) == exp).all()
        e3 = fa.VerifyEngine(0, max_txn=8192, ring_depth=2)
        try:
            assert (e3.verify_txns(arena, txns) == exp).all()
        finally:
            e3.close()
        assert (e2.verify_txns(arena, txns) == exp).all()
    finally:
        e1.close()
        e2.close()


def test_nonblocking_poll_sees_completion(engine, oracle):
    """The ring slots' completion words: a non-blocking poll returns pending
    until the batch's codes are on the host, then exactly the codes."""
    arena, txns, _ = workload.cfg1(20000, seed=0x0B02)
    exp = oracle.verify_txns(arena, txns, nthreads=8)
    for _ in range(3):
        tk = engine.submit(arena, txns)
        got = None
        for _ in range(10_000_000):
            got = engine.poll(tk, blocking=False)
            if got is not None:
                break
        assert got is not None and (got == exp).all()


@pytest.mark.parametrize("ref_mapping", [False, True])
def test_pair_kernel_path(vectors, oracle, ref_mapping):
    """FDGPU_FLAG_PAIR: two lanes per signature (fdgpu_verify_pair_kernel --
    A's and R's decode and half-size chain in adjacent lanes, the sums
    exchanged across the pair).  Held to the same bar as the one-lane
    kernel: the golden vectors under both error mappings (reference codes),
    cfg1 / cfg3 sets, the small-order x S-edge cross product, an odd batch
    (a last pair with no signature) and all-failing batches against the
    oracle; with FDGPU_FLAG_FULL_PATH as well, every lane queued by its A
    lane for the full-length kernel."""
    import firedancer_amd as fa
    key = "code_refmap" if ref_mapping else "code"
    for full in (False, True):
        eng = fa.VerifyEngine(0, max_txn=8192, ref_mapping=ref_mapping, pair=True, full_path=full)
        try:
            vs, arena, txns = _vector_batch(vectors)
            codes = eng.verify_txns(arena, txns)
            bad = [(v["src"], v["tc_id"], v[key], int(c)) for v, c in zip(vs, codes) if c != v[key]]
            assert not bad, bad[:20]
            if ref_mapping:
                continue
            sets = [workload.cfg1(2001, seed=0xA1A), workload.cfg3(600, seed=0xA1B),
                    workload.make_txns(3000, 0xA1C, corrupt=1.0, corrupt_mode=workload.MODE_R)]
            for arena, txns, _ in sets:
                got = eng.verify_txns(arena, txns)
                exp = oracle.verify_txns(arena, txns, nthreads=8)
                assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
            arena, txns = workload.pack_single(workload.small_order_cross_product())
            got = eng.verify_txns(arena, txns)
            assert (got == oracle.verify_txns(arena, txns, nthreads=8)).all()
        finally:
            eng.close()


def test_pair_auto_ring(oracle):
    """FDGPU_FLAG_PAIR_AUTO: each ring batch picks the two-lane or one-lane
    kernel by its size and how many of the engine's batches are running.
    Four batches in flight on a depth-4 ring (sizes either side of the 32 K
    cap, so both kernels run, some while others are busy) must each match
    the oracle."""
    import firedancer_amd as fa
    eng = fa.VerifyEngine(0, max_txn=40000, ring_depth=4, pair_auto=True)
    try:
        sets = [workload.cfg1(1500, seed=0xA2A), workload.cfg1(36000, seed=0xA2B),
                workload.cfg3(700, seed=0xA2C), workload.make_txns(2500, 0xA2D, corrupt=0.5)]
        tks = [eng.submit(arena, txns) for arena, txns, _ in sets]
        for tk, (arena, txns, _) in zip(tks, sets):
            got = eng.poll(tk, blocking=True)
            exp = oracle.verify_txns(arena, txns, nthreads=8)
            assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    finally:
        eng.close()


def test_spread_launch(vectors, oracle):
    """FDGPU_FLAG_SPREAD (one verify block per CU: the launch reserves the
    LDS a second block would need) with the one-lane and the two-lane
    kernel, and FDGPU_FLAG_SPREAD_AUTO with PAIR_AUTO over four ring batches
    in flight: the golden vectors' codes and the oracle's on cfg1 / cfg3
    sets.  Placement only -- the codes are the same launches'."""
    import firedancer_amd as fa
    sets = [workload.cfg1(3000, seed=0xA3A), workload.cfg3(500, seed=0xA3B)]
    for kw in (dict(spread=True), dict(spread=True, pair=True)):
        eng = fa.VerifyEngine(0, max_txn=8192, **kw)
        try:
            vs, arena, txns = _vector_batch(vectors)
            codes = eng.verify_txns(arena, txns)
            bad = [(v["src"], v["tc_id"], v["code"], int(c)) for v, c in zip(vs, codes) if c != v["code"]]
            assert not bad, (kw, bad[:20])
            for arena, txns, _ in sets:
                assert (eng.verify_txns(arena, txns) == oracle.verify_txns(arena, txns, nthreads=8)).all(), kw
        finally:
            eng.close()
    eng = fa.VerifyEngine(0, max_txn=40000, ring_depth=4, pair_auto=True, spread_auto=True)
    try:
        more = sets + [workload.cfg1(36000, seed=0xA3C), workload.make_txns(2500, 0xA3D, corrupt=0.5)]
        tks = [eng.submit(arena, txns) for arena, txns, _ in more]
        for tk, (arena, txns, _) in zip(tks, more):
            got = eng.poll(tk, blocking=True)
            assert (got == oracle.verify_txns(arena, txns, nthreads=8)).all()
    finally:
        eng.close()
