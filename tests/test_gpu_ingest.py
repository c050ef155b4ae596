"""GPU-side ingest: raw transaction payloads parsed on
the MI355X (fdt_parse.h compiled by hipcc), the signature counts scanned and
the descriptors expanded on the device, then verified.

* the device parser's output equals the host fdt_txn_parse's (itself pinned
  by test_txn_parse.c's expectations in tests/test_tile.py) byte for byte:
  footprint and fd_txn_t, on the QUIC corpus, the txn fixtures, generated
  cfg1/cfg3 txns, every single-byte mutation of two fixtures, every
  truncation, and random splices/bytes;
* the codes of a frag batch equal the oracle's on the parsed descriptors,
  payloads that do not parse get FDGPU_CODE_PARSE_FAIL, and the signature
  count produced on the device equals the host's;
* a frag batch and a descriptor batch of the same txns give the same codes.
"""
import random

import numpy as np
import pytest

from firedancer_amd import tile, workload
from firedancer_amd.ed25519 import CODE_PARSE_FAIL, FRAG_DTYPE, TXN_MAX_SZ

pytestmark = pytest.mark.gpu


def _pack(payloads):
    """payload list -> (arena with slack, frags)"""
    offs, o = [], 0
    for p in payloads:
        offs.append(o)
        o += (len(p) + 15) // 16 * 16
    arena = np.zeros(o + 256, dtype=np.uint8)
    for p, off in zip(payloads, offs):
        arena[off:off + len(p)] = np.frombuffer(p, dtype=np.uint8)
    frags = np.zeros(len(payloads), dtype=FRAG_DTYPE)
    frags["off"] = offs
    frags["sz"] = [len(p) for p in payloads]
    return arena, frags


def _payload_cases(txn_fixtures, quic_corpus):
    fx = {t["name"]: bytes.fromhex(t["payload"]) for t in txn_fixtures}
    arena, txns, _ = quic_corpus
    cases = workload.payloads(arena, txns)
    cases += list(fx.values())
    for cfgf in (workload.cfg1, workload.cfg3):
        a, tx, _ = cfgf(300, seed=5)
        cases += workload.payloads(a, tx)
    rnd = random.Random(0x1E57)
    for name in ("transaction1", "transaction2"):          # every single-byte mutation (test_txn_parse.c:141-221)
        p = fx[name]
        for i in range(len(p)):
            for off in (1, 0x7f, 0x80, 0xff) + tuple(rnd.randrange(1, 256) for _ in range(4)):
                q = bytearray(p)
                q[i] = (q[i] + off) & 255
                cases.append(bytes(q))
        cases += [p[:n] for n in range(len(p))]             # every truncation fails
    base = list(fx.values())
    for _ in range(2000):                                  # splices and random bytes
        a, b = rnd.choice(base), rnd.choice(base)
        i, j = rnd.randrange(len(a) + 1), rnd.randrange(len(b) + 1)
        cases.append(a[:i] + b[j:])
    cases += [bytes(rnd.getrandbits(8) for _ in range(rnd.choice((0, 1, 64, 200, 1232, 1233)))) for _ in range(500)]
    return cases


def test_device_parse_equals_host(engine, txn_fixtures, quic_corpus):
    cases = _payload_cases(txn_fixtures, quic_corpus)
    arena, frags = _pack(cases)
    b = engine.upload_frags(arena, frags)
    b.verify()
    b.codes()
    out, sz = b.txns()
    n_ok = 0
    for k, p in enumerate(cases):
        hsz, raw = tile.txn_parse(p)
        assert int(sz[k]) == hsz, (k, len(p))
        if hsz:
            n_ok += 1
            assert bytes(out[k, :hsz]) == raw, k
    assert n_ok > 3000 and n_ok < len(cases)
    b.free()


def test_frag_batch_codes_vs_oracle(engine, oracle, quic_corpus):
    qa, qt, qcodes = quic_corpus
    payloads = workload.payloads(qa, qt)
    ca, ct, _ = workload.cfg1(6000, seed=0xF7A6)
    payloads += workload.payloads(ca, ct)
    ma, mt, _ = workload.cfg3(1500, seed=0xF7A7)
    payloads += workload.payloads(ma, mt)
    rnd = random.Random(3)
    garbage = [bytes(rnd.getrandbits(8) for _ in range(rnd.randrange(0, 400))) for _ in range(300)]
    payloads += garbage
    rnd.shuffle(payloads)
    arena, frags = _pack(payloads)
    b = engine.upload_frags(arena, frags)
    b.verify()
    codes, sig_codes = b.codes(sig_codes=True)
    # the host's view of the same payloads: parse, descriptors, oracle codes
    parsed = [tile.txn_parse(p) for p in payloads]
    td = np.zeros(len(payloads), dtype=workload.TXN_DTYPE)
    n_sig = 0
    for k, ((fp, raw), f) in enumerate(zip(parsed, frags)):
        if not fp:
            continue
        d = tile.txn_decode(raw)
        base = int(f["off"])
        td[k] = (base + d["message_off"], int(f["sz"]) - d["message_off"], base + d["signature_off"],
                 base + d["acct_addr_off"], d["signature_cnt"])
        n_sig += d["signature_cnt"] if 1 <= d["signature_cnt"] <= 16 else 0
    ok = np.array([fp != 0 for fp, _ in parsed])
    exp = oracle.verify_txns(arena, td)
    assert (codes[~ok] == CODE_PARSE_FAIL).all()
    assert (codes[ok] == exp[ok]).all(), int((codes[ok] != exp[ok]).sum())
    assert b.n_sig == n_sig and len(sig_codes) == n_sig
    assert (codes == 0).sum() > 5000
    # the same txns as a descriptor batch (host expansion) give the same codes
    db = engine.upload(arena, td[ok])
    db.verify()
    assert (db.codes() == codes[ok]).all()
    db.free()
    b.free()


def test_frag_batch_time_and_reverify(engine):
    a, t, modes = workload.cfg1(20000, seed=0xF7A8)
    arena, frags = _pack(workload.payloads(a, t))
    b = engine.upload_frags(arena, frags)
    b.verify()
    first = b.codes().copy()
    assert ((first == 0) == (modes == 0)).all()
    wall, ingest, ver, comb = b.time2(3)
    assert ingest > 0 and ver > 0 and wall >= 0.9 * (ingest + ver)
    assert (b.codes() == first).all()
    b.free()


def test_frag_batch_edges(engine):
    # a batch of only garbage (an empty payload included), and one payload
    arena, frags = _pack([b"\x00" * 10, b""])
    b = engine.upload_frags(arena, frags)
    b.verify()
    assert (b.codes() == CODE_PARSE_FAIL).all() and b.n_sig == 0
    b.free()
    a, t, _ = workload.cfg1(1, seed=9)
    arena, frags = _pack(workload.payloads(a, t))
    b = engine.upload_frags(arena, frags)
    b.verify()
    out, sz = b.txns()
    assert sz[0] and b.codes()[0] in (0, -1, -2, -3) and out.shape == (1, TXN_MAX_SZ)
    b.free()


def test_ring_frag_batches_vs_oracle_and_trailers(engine, oracle, txn_fixtures, quic_corpus):
    """fdgpu_submit_frags / fdgpu_poll_frags (the verify tile's GPU-parse
    path through the ring slots): per frag the oracle's code on the parsed
    txn, or PARSE_FAIL; each trailer equals the host fd_txn_parse's bytes at
    the place reserved from fdt_txn_peek; a reservation other than the
    footprint gets TRAILER_CAP; several batches in flight at once."""
    from firedancer_amd.ed25519 import CODE_TRAILER_CAP, FRAG_EX_DTYPE
    cases = _payload_cases(txn_fixtures, quic_corpus)
    rnd = random.Random(0x7A11)
    rnd.shuffle(cases)
    chunks = [cases[i:i + 2500] for i in range(0, 7500, 2500)]
    def submit(ci, ps):
        arena, fr = _pack(ps)
        fx = np.zeros(len(ps), dtype=FRAG_EX_DTYPE)
        fx["off"], fx["sz"] = fr["off"], fr["sz"]
        tr = 0
        caps = []
        for k, p in enumerate(ps):
            fp, _ = tile.txn_peek(p)
            if ci == 2 and k % 97 == 5 and fp:
                fp += 10                                      # a wrong reservation
            fx[k]["tr_off"], fx[k]["tr_cap"] = tr, fp
            caps.append(fp)
            tr += (fp + 3) & ~3
        return engine.submit_frags(arena, fx, tr), arena, fx, ps

    inflight = [submit(0, chunks[0]), submit(1, chunks[1])]     # both ring slots busy
    for ci in range(len(chunks)):
        tk, arena, fx, ps = inflight.pop(0)
        codes, trailers = engine.poll_frags(tk)
        if ci + 2 < len(chunks):
            inflight.append(submit(ci + 2, chunks[ci + 2]))
        td = np.zeros(len(ps), dtype=workload.TXN_DTYPE)
        parsed = [tile.txn_parse(p) for p in ps]
        for k, ((fp, raw), f) in enumerate(zip(parsed, fx)):
            if fp:
                d = tile.txn_decode(raw)
                base = int(f["off"])
                td[k] = (base + d["message_off"], int(f["sz"]) - d["message_off"], base + d["signature_off"],
                         base + d["acct_addr_off"], d["signature_cnt"])
        exp = oracle.verify_txns(arena, td)
        for k, ((fp, raw), f) in enumerate(zip(parsed, fx)):
            if not fp:
                assert codes[k] == CODE_PARSE_FAIL, k
            elif int(f["tr_cap"]) != fp:
                assert codes[k] == CODE_TRAILER_CAP, k
            else:
                assert codes[k] == exp[k], k
                o = int(f["tr_off"])
                assert bytes(trailers[o:o + fp]) == raw, k
        if ci == 2:
            assert (codes == CODE_TRAILER_CAP).sum() > 5


def _aligned(n, a=4096):
    buf = np.zeros(n + a, dtype=np.uint8)
    o = (-buf.ctypes.data) % a
    return buf[o:o + n]


def test_ring_frag_io_batches(engine, oracle, txn_fixtures, quic_corpus):
    """fdgpu_submit_frags_io / fdgpu_poll_frags_io (the verify tile's gather
    path): payloads at 64-B chunk offsets of a registered "in dcache", read
    there by the device; per frag the oracle's code or PARSE_FAIL, the dedup
    tag fd_hash(seed, first signature, 64) as the host computes it, and the
    out frag [payload][pad][fd_txn_t][u16 sz] written at its reserved place
    in a registered "out dcache", byte-equal to the host layout; a
    reservation too small for the parsed out frag gets TRAILER_CAP; two
    batches in flight; a payload outside every registered region is
    refused."""
    from firedancer_amd.ed25519 import CODE_TRAILER_CAP, FRAG_IO_DTYPE
    from firedancer_amd import _lib
    L = _lib.lib()
    cases = [p for p in _payload_cases(txn_fixtures, quic_corpus) if len(p) <= 1232]
    rnd = random.Random(0x10A)
    rnd.shuffle(cases)
    chunks = [cases[i:i + 2500] for i in range(0, 7500, 2500)]
    seed = 0x5EED1234ABCD
    in_buf = _aligned(sum((len(p) + 63) // 64 * 64 for p in cases[:7500]) + 4096)
    out_buf = _aligned(7500 * (1232 + 852 + 64) + 4096)
    engine.host_register(in_buf)
    engine.host_register(out_buf)
    try:
        in_off = [0]
        out_base = [0]

        def submit(ci, ps):
            fio = np.zeros(len(ps), dtype=FRAG_IO_DTYPE)
            o = 0
            short = set()
            for k, p in enumerate(ps):
                a = in_off[0]
                in_buf[a:a + len(p)] = np.frombuffer(p, dtype=np.uint8)
                in_off[0] = a + (len(p) + 63) // 64 * 64
                cap = L.fdgpu_frag_out_cap(len(p))
                fp, _ = tile.txn_parse(p)
                if ci == 1 and k % 89 == 3 and fp:
                    cap = ((len(p) + 1) & ~1) + fp + 1        # one byte short
                    short.add(k)
                fio[k] = (in_buf.ctypes.data + a, len(p), o, cap, 0, 0)
                o += (cap + 63) // 64 * 64
            base = out_base[0]
            out_base[0] += o
            view = out_buf[base:base + o]
            return engine.submit_frags_io(fio, view, o, seed), fio, view, ps, short

        inflight = [submit(0, chunks[0]), submit(1, chunks[1])]
        for ci in range(len(chunks)):
            tk, fio, view, ps, short = inflight.pop(0)
            codes, tags, osz = engine.poll_frags_io(tk)
            if ci + 2 < len(chunks):
                inflight.append(submit(ci + 2, chunks[ci + 2]))
            arena = np.frombuffer(b"".join(ps) + b"\0" * 16, dtype=np.uint8)
            offs = np.cumsum([0] + [len(p) for p in ps])
            td = np.zeros(len(ps), dtype=workload.TXN_DTYPE)
            parsed = [tile.txn_parse(p) for p in ps]
            for k, (fp, raw) in enumerate(parsed):
                if fp:
                    d = tile.txn_decode(raw)
                    b0 = int(offs[k])
                    td[k] = (b0 + d["message_off"], len(ps[k]) - d["message_off"], b0 + d["signature_off"],
                             b0 + d["acct_addr_off"], d["signature_cnt"])
            exp = oracle.verify_txns(arena, td)
            for k, ((fp, raw), f) in enumerate(zip(parsed, fio)):
                p = ps[k]
                if not fp:
                    assert codes[k] == CODE_PARSE_FAIL and osz[k] == 0 and tags[k] == 0, k
                    continue
                d = tile.txn_decode(raw)
                so = d["signature_off"]
                assert tags[k] == tile.fd_hash(seed, p[so:so + 64]), k
                if k in short:
                    assert codes[k] == CODE_TRAILER_CAP and osz[k] == 0, k
                    continue
                assert codes[k] == exp[k], k
                frag = p + b"\0" * (((len(p) + 1) & ~1) - len(p)) + raw + len(p).to_bytes(2, "little")
                assert osz[k] == len(frag), k
                o = int(f["out_off"])
                assert bytes(view[o:o + len(frag)]) == frag, k
            if ci == 1:
                assert len(short) > 5
        # a payload outside every registered region
        stray = np.zeros(4096, dtype=np.uint8)
        fio = np.zeros(1, dtype=FRAG_IO_DTYPE)
        fio[0] = ((stray.ctypes.data + 63) // 64 * 64, 100, 0, L.fdgpu_frag_out_cap(100), 0, 0)
        with pytest.raises(RuntimeError, match=r"\(-14\)"):          # FDGPU_ERR_UNREG: a wiring error
            engine.submit_frags_io(fio, out_buf, 4096, seed)
    finally:
        engine.host_unregister(in_buf)
        engine.host_unregister(out_buf)


def _pages(n):
    """n bytes on pages of their own (registrable next to other buffers)"""
    return _aligned((n + 4095) // 4096 * 4096)[:n]


def test_frag_io_device_lap_recheck(engine, oracle):
    """The gather's overrun re-check on the device (fdgpu_submit_frags_io
    with links: the reference's seq re-check after its copy,
    fd_mux.c:641-655): after reading a payload the device re-reads the frag's
    line in the registered in mcache; a line that holds another seq (the
    producer republished it) gives FDGPU_CODE_LAPPED, no tag and no out frag;
    every other frag -- including one naming no link, which is not
    re-checked -- verifies as the oracle says and gets its out frag.  A link
    index outside the table, an unregistered mcache or a bad depth is
    refused."""
    from firedancer_amd.ed25519 import CODE_LAPPED, FRAG_IO_DTYPE
    from firedancer_amd import _lib
    L = _lib.lib()
    a, t, _ = workload.cfg1(310, seed=0x1A9)
    ps = [p for p in workload.payloads(a, t) if tile.txn_parse(p)[0]][:300]
    assert len(ps) == 300
    depth, seq0 = 256, (1 << 40) + 7
    mc = _pages(depth * 32).view(tile.FRAG_META_DTYPE)
    in_buf = _pages(len(ps) * 1280)
    out_buf = _pages(len(ps) * 2176)
    for b in (mc, in_buf, out_buf):
        engine.host_register(b)
    try:
        fio = np.zeros(len(ps), dtype=FRAG_IO_DTYPE)
        o = 0
        for k, p in enumerate(ps):
            in_buf[k * 1280:k * 1280 + len(p)] = np.frombuffer(p, dtype=np.uint8)
            cap = L.fdgpu_frag_out_cap(len(p))
            fio[k] = (in_buf.ctypes.data + k * 1280, len(p), o, cap, 0 if k % 50 == 7 else 1, seq0 + k)
            o += (cap + 63) // 64 * 64
            mc[(seq0 + k) % depth]["seq"] = seq0 + k
        lapped = set(range(3, len(ps), 11)) - {k for k in range(len(ps)) if k % 50 == 7} - set(range(depth, len(ps)))
        for k in range(len(ps)):
            if k >= depth:                                 # lines reused by later frags of the batch: seq0 + k
                continue
            if k in lapped:
                mc[(seq0 + k) % depth]["seq"] = seq0 + k + depth
        # frags past depth share lines with the first ones: the line holds the later seq, so the earlier
        # frag of each such pair is lapped and the later one is not
        lapped |= {k - depth for k in range(depth, len(ps)) if (k - depth) % 50 != 7}
        for k in range(depth, len(ps)):
            mc[(seq0 + k) % depth]["seq"] = seq0 + k
        links = [(mc.ctypes.data, depth)]
        tk = engine.submit_frags_io(fio, out_buf, o, 0x77, links=links)
        codes, tags, osz = engine.poll_frags_io(tk)
        arena = np.frombuffer(b"".join(ps) + b"\0" * 16, dtype=np.uint8)
        offs = np.cumsum([0] + [len(p) for p in ps])
        td = np.zeros(len(ps), dtype=workload.TXN_DTYPE)
        for k, p in enumerate(ps):
            d = tile.txn_decode(tile.txn_parse(p)[1])
            td[k] = (int(offs[k]) + d["message_off"], len(p) - d["message_off"], int(offs[k]) + d["signature_off"],
                     int(offs[k]) + d["acct_addr_off"], d["signature_cnt"])
        exp = oracle.verify_txns(arena, td)
        assert len(lapped) > 20
        for k, p in enumerate(ps):
            if k in lapped:
                assert codes[k] == CODE_LAPPED and tags[k] == 0 and osz[k] == 0, k
            else:
                assert codes[k] == exp[k] and osz[k] > len(p), k
                fp, raw = tile.txn_parse(p)
                frag = p + b"\0" * (((len(p) + 1) & ~1) - len(p)) + raw + len(p).to_bytes(2, "little")
                off = int(fio[k]["out_off"])
                assert bytes(out_buf[off:off + len(frag)]) == frag, k
        bad = fio[:4].copy()
        bad["link"] = 2                                    # only one link given
        with pytest.raises(RuntimeError):
            engine.submit_frags_io(bad, out_buf, o, 0x77, links=links)
        stray = _pages(depth * 32)
        with pytest.raises(RuntimeError):
            engine.submit_frags_io(fio[:4], out_buf, o, 0x77, links=[(stray.ctypes.data, depth)])
        with pytest.raises(RuntimeError):
            engine.submit_frags_io(fio[:4], out_buf, o, 0x77, links=[(mc.ctypes.data, depth - 1)])
    finally:
        for b in (mc, in_buf, out_buf):
            engine.host_unregister(b)


def test_frag_io_pair_kernel(oracle):
    """Gathered frag batches through an engine with FDGPU_FLAG_PAIR: the
    signature count comes from the device (parse + expand), the pair kernel
    sizes its grid from the bound -- codes equal the oracle's on cfg1 and
    cfg3 payloads."""
    import firedancer_amd as fa
    from firedancer_amd import _lib
    L = _lib.lib()
    eng = fa.VerifyEngine(0, max_txn=4096, pair=True)
    try:
        for gen, seed in ((workload.cfg1, 0xB1), (workload.cfg3, 0xB2)):
            a, t, _ = gen(1500, seed=seed)
            ps = [p for p in workload.payloads(a, t) if tile.txn_parse(p)[0]]
            in_buf, out_buf = _pages(len(ps) * 1280), _pages(len(ps) * 2176)
            eng.host_register(in_buf)
            eng.host_register(out_buf)
            try:
                fio = np.zeros(len(ps), dtype=tile.FRAG_IO_DTYPE)
                o = 0
                for k, p in enumerate(ps):
                    in_buf[k * 1280:k * 1280 + len(p)] = np.frombuffer(p, dtype=np.uint8)
                    cap = L.fdgpu_frag_out_cap(len(p))
                    fio[k] = (in_buf.ctypes.data + k * 1280, len(p), o, cap, 0, 0)
                    o += (cap + 63) // 64 * 64
                codes, _, _ = eng.poll_frags_io(eng.submit_frags_io(fio, out_buf, o, 0x33))
                arena = np.frombuffer(b"".join(ps) + b"\0" * 16, dtype=np.uint8)
                offs = np.cumsum([0] + [len(p) for p in ps])
                td = np.zeros(len(ps), dtype=workload.TXN_DTYPE)
                for k, p in enumerate(ps):
                    d = tile.txn_decode(tile.txn_parse(p)[1])
                    td[k] = (int(offs[k]) + d["message_off"], len(p) - d["message_off"],
                             int(offs[k]) + d["signature_off"], int(offs[k]) + d["acct_addr_off"], d["signature_cnt"])
                assert (codes == oracle.verify_txns(arena, td, nthreads=8)).all()
            finally:
                eng.host_unregister(in_buf)
                eng.host_unregister(out_buf)
    finally:
        eng.close()


@pytest.mark.gpu
def test_frag_io_merged_verify(oracle):
    """FDGPU_FLAG_MERGE: gathered batches submitted back to back have their
    verifies merged into shared launches (one block row per batch) on the
    engine's merge streams, launched from submit and poll calls.  Four
    batches (cfg1 and cfg3 payloads, different sizes) in flight at once,
    polled non-blocking, blocking and out of order: codes, tags, out sizes
    and every out-frag byte equal those of an engine without the flag, and
    the codes equal the oracle's."""
    import firedancer_amd as fa
    from firedancer_amd import _lib
    L = _lib.lib()
    sets = []
    for gen, n, seed in ((workload.cfg1, 1800, 0xC1), (workload.cfg3, 400, 0xC2), (workload.cfg1, 700, 0xC3),
                         (workload.cfg3, 900, 0xC4)):
        a, t, _ = gen(n, seed=seed)
        sets.append([p for p in workload.payloads(a, t) if tile.txn_parse(p)[0]])
    results = {}
    for merge in (False, True):
        eng = fa.VerifyEngine(0, max_txn=2048, ring_depth=4, merge=merge)
        bufs = []
        try:
            tks = []
            for ps in sets:
                in_buf, out_buf = _pages(len(ps) * 1280), _pages(len(ps) * 2176)
                eng.host_register(in_buf)
                eng.host_register(out_buf)
                bufs += [in_buf, out_buf]
                fio = np.zeros(len(ps), dtype=tile.FRAG_IO_DTYPE)
                o = 0
                for k, p in enumerate(ps):
                    in_buf[k * 1280:k * 1280 + len(p)] = np.frombuffer(p, dtype=np.uint8)
                    cap = L.fdgpu_frag_out_cap(len(p))
                    fio[k] = (in_buf.ctypes.data + k * 1280, len(p), o, cap, 0, 0)
                    o += (cap + 63) // 64 * 64
                tks.append((eng.submit_frags_io(fio, out_buf, o, 0x44), out_buf, o))
            res = [None] * len(tks)
            for j in (2, 0):                                  # blocking, out of order (2 may still wait to merge)
                res[j] = eng.poll_frags_io(tks[j][0], blocking=True)
            for j in (3, 1):                                  # non-blocking until done
                r = None
                while r is None:
                    r = eng.poll_frags_io(tks[j][0], blocking=False)
                res[j] = r
            results[merge] = [(c.copy(), tg.copy(), sz.copy(), bytes(ob[:o])) for (c, tg, sz), (_, ob, o) in zip(res, tks)]
        finally:
            for b in bufs:
                eng.host_unregister(b)
            eng.close()
    for j, ps in enumerate(sets):
        (c0, t0, s0, o0), (c1, t1, s1, o1) = results[False][j], results[True][j]
        assert (c0 == c1).all() and (t0 == t1).all() and (s0 == s1).all() and o0 == o1, j
        arena = np.frombuffer(b"".join(ps) + b"\0" * 16, dtype=np.uint8)
        offs = np.cumsum([0] + [len(p) for p in ps])
        td = np.zeros(len(ps), dtype=workload.TXN_DTYPE)
        for k, p in enumerate(ps):
            d = tile.txn_decode(tile.txn_parse(p)[1])
            td[k] = (int(offs[k]) + d["message_off"], len(p) - d["message_off"],
                     int(offs[k]) + d["signature_off"], int(offs[k]) + d["acct_addr_off"], d["signature_cnt"])
        assert (c1 == oracle.verify_txns(arena, td, nthreads=8)).all(), j


def test_frag_io_dma_gather_and_small_grids():
    """The gathered path's two other shapes, in a child process (both are read
    once at library load): FDGPU_IO_DMA=1 -- the payload ranges copied by the
    DMA engines into the slot's mirror and parsed, re-checked and verified
    there -- and the ingest / finish kernels on one block each (every wave
    strides over many 64-frag groups).  Each runs the gathered-batch tests
    above: codes, tags and out frags against the oracle, and the lap re-check."""
    import os
    import subprocess
    import sys
    if os.environ.get("FDGPU_IO_SUBRUN"):
        pytest.skip("inside the child run")
    here = os.path.dirname(os.path.abspath(__file__))
    for extra in ({"FDGPU_IO_DMA": "1"}, {"FDGPU_AUX_BLOCKS_IN": "1", "FDGPU_AUX_BLOCKS_FIN": "1"}):
        env = dict(os.environ, FDGPU_IO_SUBRUN="1", **extra)
        r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "gpu",
                            os.path.join(here, "test_gpu_ingest.py"), "-k", "frag_io"],
                           env=env, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, (extra, r.stdout[-3000:], r.stderr[-2000:])
        assert " passed" in r.stdout, r.stdout[-2000:]


@pytest.mark.gpu
def test_frag_io_failed_merge_then_good_batch(oracle, monkeypatch):
    """a gathered batch whose merged verify fails after its
    ingest was queued (injected: FDGPU_DEBUG_FAIL_MERGE=1) leaves the slot's
    device-side signature count behind; the poll reports the failure (the
    submit returns the ticket), and the next batch on the same slot -- one
    ring slot, so it is the same one -- clears the count first: its codes equal
    the oracle's."""
    import firedancer_amd as fa
    from firedancer_amd import _lib
    L = _lib.lib()
    monkeypatch.setenv("FDGPU_DEBUG_FAIL_MERGE", "1")
    eng = fa.VerifyEngine(0, max_txn=2048, ring_depth=1, merge=True)
    monkeypatch.delenv("FDGPU_DEBUG_FAIL_MERGE")
    bufs = []
    try:
        outs = []
        for seed in (0xD1, 0xD2):
            a, t, _ = workload.cfg1(1500, seed=seed)
            ps = [p for p in workload.payloads(a, t) if tile.txn_parse(p)[0]]
            in_buf, out_buf = _pages(len(ps) * 1280), _pages(len(ps) * 2176)
            eng.host_register(in_buf)
            eng.host_register(out_buf)
            bufs += [in_buf, out_buf]
            fio = np.zeros(len(ps), dtype=tile.FRAG_IO_DTYPE)
            o = 0
            for k, p in enumerate(ps):
                in_buf[k * 1280:k * 1280 + len(p)] = np.frombuffer(p, dtype=np.uint8)
                cap = L.fdgpu_frag_out_cap(len(p))
                fio[k] = (in_buf.ctypes.data + k * 1280, len(p), o, cap, 0, 0)
                o += (cap + 63) // 64 * 64
            outs.append((ps, fio, out_buf, o))
        ps, fio, out_buf, o = outs[0]
        tk = eng.submit_frags_io(fio, out_buf, o, 0x55)          # its merge fails: a ticket all the same
        with pytest.raises(RuntimeError):
            eng.poll_frags_io(tk, blocking=True)
        ps, fio, out_buf, o = outs[1]
        codes, _, _ = eng.poll_frags_io(eng.submit_frags_io(fio, out_buf, o, 0x55), blocking=True)
        arena = np.frombuffer(b"".join(ps) + b"\0" * 16, dtype=np.uint8)
        offs = np.cumsum([0] + [len(p) for p in ps])
        td = np.zeros(len(ps), dtype=workload.TXN_DTYPE)
        for k, p in enumerate(ps):
            d = tile.txn_decode(tile.txn_parse(p)[1])
            td[k] = (int(offs[k]) + d["message_off"], len(p) - d["message_off"],
                     int(offs[k]) + d["signature_off"], int(offs[k]) + d["acct_addr_off"], d["signature_cnt"])
        assert (codes == oracle.verify_txns(arena, td, nthreads=8)).all()
    finally:
        for b in bufs:
            eng.host_unregister(b)
        eng.close()
