"""Verify-stage integration on CPU: tango wire
formats, tcache, fd_hash, fd_txn_parse and the verify / dedup tiles, checked
against the reference's own test expectations (test_txn_parse.c,
test_tcache.c, test_verify.c) and against sequential models of the reference
loops.  The verify tiles here run over a PyVerifier whose verdicts come from
the CPU oracle (the GPU engine is exercised by test_tile_gpu.py)."""
import ctypes
import hashlib
import os
import random

import numpy as np
import pytest

from firedancer_amd import tile, workload
import tile_model


@pytest.fixture(scope="module")
def fixtures(txn_fixtures):
    return {t["name"]: bytes.fromhex(t["payload"]) for t in txn_fixtures}


def oracle_fn(oracle):
    return lambda arena, txns: oracle.verify_txns(arena, txns)


# ------------------------------------------------------------------ hash

def test_fd_hash_is_xxh64():
    """fd_hash (src/util/fd_hash.c, xxhash-r39) is XXH64: pinned against the
    independent xxhash package for every tail length and several seeds."""
    import xxhash
    rnd = random.Random(7)
    for n in list(range(0, 80)) + [127, 128, 1232]:
        for seed in (0, 1, 2**63 + 5, rnd.getrandbits(64)):
            d = bytes(rnd.getrandbits(8) for _ in range(n))
            assert tile.fd_hash(seed, d) == xxhash.xxh64_intdigest(d, seed=seed), (n, seed)


# ---------------------------------------------------------------- tcache

def test_tcache_params():
    """test_tcache.c:14-40 expectations."""
    L = tile.lib()
    assert L.fdt_tcache_footprint(1, 4) == 128
    assert not L.fdt_tcache_footprint(2**64 - 1, 4)
    assert not L.fdt_tcache_footprint(1, 2**64 - 1)
    assert [L.fdt_tcache_map_cnt_default(d) for d in (0, 1, 2, 3, 6, 7)] == [0, 8, 8, 16, 16, 32]
    rnd = random.Random(3)
    for _ in range(20000):
        depth = rnd.randrange(1024)
        map_cnt = (1 << rnd.randrange(16)) + rnd.choice((-1, 0, 1))
        fp = L.fdt_tcache_footprint(depth, map_cnt)
        mc = map_cnt or L.fdt_tcache_map_cnt_default(depth)
        if depth == 0 or mc < depth + 2 or (mc & (mc - 1)):
            assert fp == 0
        else:
            assert fp == ((4 + depth + mc) * 8 + 127) // 128 * 128


@pytest.mark.parametrize("depth,map_cnt", [(16, 64), (1, 4), (100, 0), (1000, 2048)])
def test_tcache_vs_model(depth, map_cnt):
    """Random insert/query mix with heavy temporally-local duplication vs the
    ring+set model: same dup answers, map == ring contents, ring order."""
    tc = tile.TCache(depth, map_cnt)
    model = tile_model.TCacheModel(depth)
    rnd = random.Random(depth)
    recent = []
    for i in range(30000):
        if recent and rnd.random() < 0.5:
            tag = recent[-1 - min(int(rnd.expovariate(1 / max(depth, 1))), len(recent) - 1)]
        else:
            tag = rnd.getrandbits(64) or 1
            if rnd.random() < 0.3:                      # force probe collisions
                tag = (tag & ~(tc.map_cnt - 1)) | rnd.randrange(4)
        recent.append(tag)
        if rnd.random() < 0.2:
            assert tc.query(tag) == model.query(tag)
        else:
            assert tc.insert(tag) == model.insert(tag), i
    w = tc.words()
    ring, mp = w[4:4 + depth], w[4 + depth:]
    assert set(int(x) for x in mp if x) == model.set
    oldest = int(w[3])
    order = [int(x) for x in np.roll(ring, -oldest) if x]
    assert order == list(model.ring)


def test_tcache_reset():
    tc = tile.TCache(16, 64)
    for t in range(1, 40):
        tc.insert(t)
    tc.reset()
    assert not any(tc.query(t) for t in range(1, 40))
    assert not tc.words()[3:].any()


# ----------------------------------------------------------------- tango

def test_mcache_publish_poll_overrun():
    lk = tile.Link(depth=8, mtu=1232, seq0=100)
    rc, meta, found = lk.poll(100)
    assert rc == 0 and found == 99                        # line initialised to seq-1
    seqs = [lk.publish(bytes([i]) * (i + 1), sig=1000 + i) for i in range(5)]
    assert seqs == list(range(100, 105))
    for i, s in enumerate(seqs):
        rc, meta, _ = lk.poll(s)
        assert rc == 1 and meta["sig"] == 1000 + i and meta["sz"] == i + 1
        assert lk.payload(meta) == bytes([i]) * (i + 1)
        assert meta["ctl"] == tile.frag_meta_ctl(0, 1, 1, 0) == 3
    for i in range(5, 12):
        lk.publish(b"x", sig=i)
    rc, meta, found = lk.poll(101)                       # overwritten by seq 109
    assert rc == -1 and found == 109
    assert tile.frag_meta_ctl(5, 0, 1, 1) == (5 << 3) | 6


def test_dcache_compact_ring():
    """fd_dcache.h:262-269: advance by whole chunk pairs, wrap past wmark,
    frags never straddle the end of the data region."""
    lk = tile.Link(depth=16, mtu=1232)
    cmtu = tile.lib().fdt_dcache_chunk_mtu(1232)
    assert cmtu == 20 and lk.wmark == lk.chunk1 - cmtu
    assert tile.dcache_compact_next(0, 1, 0, 100) == 2
    assert tile.dcache_compact_next(0, 128, 0, 100) == 2
    assert tile.dcache_compact_next(0, 129, 0, 100) == 4
    assert tile.dcache_compact_next(98, 64, 0, 100) == 100
    assert tile.dcache_compact_next(100, 64, 0, 100) == 0
    rnd = random.Random(1)
    ch = 0
    for _ in range(2000):
        sz = rnd.randrange(1, 1233)
        assert ch <= lk.wmark and (ch + (sz + 63) // 64) <= lk.chunk1
        ch = tile.dcache_compact_next(ch, sz, 0, lk.wmark)


# ------------------------------------------------------------ txn parse

def test_txn_parse_transaction1(fixtures):
    """test_txn_parse.c:34-80"""
    p = fixtures["transaction1"]
    ctr = tile.ParseCounters()
    sz, raw = tile.txn_parse(p, ctr)
    assert sz and ctr.success_cnt == 1 and ctr.failure_cnt == 0
    d = tile.txn_decode(raw)
    assert d["transaction_version"] == tile.TXN_VLEGACY and d["signature_cnt"] == 4
    assert [p[d["signature_off"] + 64 * j] for j in range(4)] == [97, 189, 11, 108]
    assert d["message_off"] == d["signature_off"] + 4 * 64
    assert (d["readonly_signed_cnt"], d["readonly_unsigned_cnt"], d["acct_addr_cnt"]) == (1, 11, 23)
    assert [p[d["acct_addr_off"] + 32 * j] for j in range(23)] == [
        220, 255, 85, 89, 201, 170, 194, 48, 228, 123, 151, 133, 6, 6, 203, 6, 11, 6, 0, 140, 3, 5, 168]
    assert p[d["recent_blockhash_off"]] == 155
    assert (d["addr_table_lookup_cnt"], d["addr_table_adtl_writable_cnt"], d["addr_table_adtl_cnt"]) == (0, 0, 0)
    assert d["instr_cnt"] == 7
    ix = d["instr"]
    assert (ix[0]["program_id"], ix[0]["acct_cnt"], ix[0]["data_sz"]) == (20, 0, 5)
    assert p[ix[0]["data_off"]:ix[0]["data_off"] + 5] == bytes([0x00, 0xE0, 0x93, 0x04, 0x00])
    assert (ix[1]["program_id"], ix[1]["acct_cnt"], ix[1]["data_sz"]) == (18, 2, 12)
    assert (p[ix[1]["acct_off"]], p[ix[1]["data_off"]]) == (0, 2)
    assert (ix[6]["program_id"], ix[6]["acct_cnt"], ix[6]["data_sz"]) == (22, 21, 12)
    assert (p[ix[6]["acct_off"]], p[ix[6]["data_off"]]) == (14, 211)


def test_txn_parse_transaction2(fixtures):
    """test_txn_parse.c:82-139 (v0 with address lookup tables)"""
    p = fixtures["transaction2"]
    sz, raw = tile.txn_parse(p)
    d = tile.txn_decode(raw)
    assert d["transaction_version"] == tile.TXN_V0 and d["signature_cnt"] == 1
    assert (d["readonly_signed_cnt"], d["readonly_unsigned_cnt"], d["acct_addr_cnt"]) == (0, 2, 6)
    assert p[d["recent_blockhash_off"]] == 148
    assert (d["addr_table_lookup_cnt"], d["addr_table_adtl_writable_cnt"], d["addr_table_adtl_cnt"]) == (3, 12, 21)
    ix = d["instr"]
    assert (ix[0]["program_id"], ix[0]["acct_cnt"], ix[0]["data_sz"]) == (4, 0, 5)
    assert (ix[1]["program_id"], ix[1]["acct_cnt"], ix[1]["data_sz"]) == (5, 39, 38)
    assert (p[ix[1]["acct_off"]], p[ix[1]["data_off"]]) == (18, 229)
    lut = d["luts"]
    assert (p[lut[0]["addr_off"]], lut[0]["writable_cnt"], lut[0]["readonly_cnt"]) == (54, 4, 4)
    assert p[lut[0]["readonly_off"] + 1] == 117
    assert (p[lut[1]["addr_off"]], lut[1]["writable_cnt"], lut[1]["readonly_cnt"]) == (34, 4, 4)
    assert (p[lut[1]["writable_off"]], p[lut[1]["readonly_off"]]) == (196, 194)
    assert (p[lut[2]["addr_off"]], lut[2]["writable_cnt"], lut[2]["readonly_cnt"]) == (212, 4, 1)
    assert (p[lut[2]["writable_off"]], p[lut[2]["readonly_off"]]) == (91, 97)
    assert sz == tile.lib().fdt_txn_footprint(2, 3)


def test_txn_parse_fixture_footprints(fixtures):
    """test_txn_parse.c:254-260"""
    L = tile.lib()
    assert tile.txn_parse(fixtures["transaction3"])[0] == tile.TXN_MAX_SZ
    assert tile.txn_parse(fixtures["transaction4"])[0] == 20
    assert tile.txn_parse(fixtures["transaction5"])[0] == 0
    assert tile.txn_parse(fixtures["transaction6"])[0] == L.fdt_txn_footprint(1, 0)


@pytest.mark.parametrize("name", ["transaction1", "transaction2"])
def test_txn_parse_mutations(fixtures, name):
    """test_txn_parse.c:141-221: every truncation fails; every single-byte
    mutation parses iff the byte stays within the field's legal range, and
    mutations of free bytes leave the parsed struct identical."""
    import ctypes
    L = tile.lib()
    p = bytearray(fixtures[name])
    n = len(p)
    sz, raw = tile.txn_parse(bytes(p))
    d = tile.txn_decode(raw)
    lo, hi = list(p), list(p)

    def ok(start, ln):
        for k in range(start, start + ln):
            lo[k], hi[k] = 0, 255

    ok(d["signature_off"], 64 * d["signature_cnt"])
    ok(d["acct_addr_off"], 32 * d["acct_addr_cnt"])
    ok(d["recent_blockhash_off"], 32)
    ro = d["message_off"] + (2 if d["transaction_version"] == tile.TXN_V0 else 1)
    lo[ro], hi[ro] = 0, d["signature_cnt"] - 1
    lo[ro + 1], hi[ro + 1] = 0, d["acct_addr_cnt"] - d["signature_cnt"]
    total = d["acct_addr_cnt"] + d["addr_table_adtl_cnt"]
    for ins in d["instr"]:
        lo[ins["acct_off"] - 2], hi[ins["acct_off"] - 2] = 1, d["acct_addr_cnt"] - 1
        ok(ins["data_off"], ins["data_sz"])
        for k in range(ins["data_sz"]):
            p[ins["data_off"] + k] = 0xDA
        for k in range(ins["acct_cnt"]):
            lo[ins["acct_off"] + k], hi[ins["acct_off"] + k] = 0, total - 1
            p[ins["acct_off"] + k] = (total - 1 - k) % total
    for lut in d["luts"]:
        ok(lut["addr_off"], 32)
        ok(lut["writable_off"], lut["writable_cnt"])
        ok(lut["readonly_off"], lut["readonly_cnt"])
    sz2, raw2 = tile.txn_parse(bytes(p))
    assert sz2 == sz and raw2 == raw
    buf = ctypes.create_string_buffer(tile.TXN_MAX_SZ + 16)
    ctr = tile.ParseCounters()
    pb = (ctypes.c_uint8 * n).from_buffer(p)
    for i in range(n):
        assert L.fdt_txn_parse(pb, i, buf, ctypes.byref(ctr)) == 0
        orig = p[i]
        for off in range(1, 256):
            p[i] = (orig + off) & 255
            got = L.fdt_txn_parse(pb, n, buf, ctypes.byref(ctr))
            if lo[i] == 0 and hi[i] == 255:
                assert got == sz and buf.raw[:sz] == raw, (i, off)
            elif p[i] < lo[i] or p[i] > hi[i]:
                assert got == 0, (i, off)
            else:
                assert got, (i, off)
        p[i] = orig
    assert ctr.success_cnt and ctr.failure_cnt and ctr.success_cnt + ctr.failure_cnt == 256 * n
    assert all(ctr.failure_ring[k] for k in range(32))


def test_txn_parse_corpora_offsets(quic_corpus, fixtures):
    """Every QUIC-corpus txn and generated txn parses, and the parsed
    offsets are the ones the golden descriptors hold."""
    arena, txns, codes = quic_corpus
    for t in txns[:1000]:
        p = bytes(arena[int(t["sig_off"]) - 1: int(t["msg_off"]) + int(t["msg_sz"])])
        sz, raw = tile.txn_parse(p)
        assert sz
        mo, ms, so, po, sc = tile_model.txn_descriptor(p, raw)
        base = int(t["sig_off"]) - 1
        assert (mo + base, ms, so + base, po + base, sc) == tuple(int(x) for x in t)
    for cfgf in (workload.cfg1, workload.cfg3):
        a, tx, _ = cfgf(200, seed=11)
        for p in workload.payloads(a, tx):
            assert tile.txn_parse(p)[0]


def test_txn_parse_rejects_malformed():
    """compact-u16 minimal encoding and trailing bytes (fd_compact_u16.h:60-75, fd_txn_parse.c:221)."""
    a, tx, _ = workload.cfg1(4, seed=2)
    p = workload.payloads(a, tx)[0]
    assert tile.txn_parse(p)[0]
    assert tile.txn_parse(p + b"\0")[0] == 0                       # trailing byte
    assert tile.txn_parse(p[:-1])[0] == 0
    sz, raw = tile.txn_parse(p)
    d = tile.txn_decode(raw)
    i = d["message_off"] + 3                                        # acct_addr_cnt compact-u16
    bad = p[:i] + bytes([p[i] | 0x80, 0x00]) + p[i + 1:]            # non-minimal 2-byte form
    assert tile.txn_parse(bad)[0] == 0
    assert tile.txn_parse(b"")[0] == 0 and tile.txn_parse(b"\0" * 1233)[0] == 0


def test_txn_parse_random_bytes(fixtures):
    """fd_txn_parse on untrusted bytes: random payloads of every size class,
    random splices of the fixtures and every truncation of one fixture never
    read or write out of bounds (run under ASan/UBSan by test_sanitize.py) and
    accept only what round-trips through the restated decoder."""
    rnd = random.Random(0xF022)
    base = list(fixtures.values())
    cases = [bytes(rnd.getrandbits(8) for _ in range(rnd.choice((0, 1, 3, 64, 65, 200, 1231, 1232, 1233, 2000))))
             for _ in range(1500)]
    for _ in range(1500):
        a, b = rnd.choice(base), rnd.choice(base)
        i, j = rnd.randrange(len(a) + 1), rnd.randrange(len(b) + 1)
        cases.append(a[:i] + b[j:])
    p = base[0]
    cases += [p[:n] for n in range(len(p) + 1)]
    for cse in cases:
        sz, raw = tile.txn_parse(cse)
        if sz:
            d = tile.txn_decode(raw)
            assert d["signature_off"] + 64 * d["signature_cnt"] <= len(cse)
            assert d["message_off"] < len(cse) or len(cse) == 0


# ----------------------------------------------------------- verify tile

def _run_tile(payloads, verifier, seed=0xABCD, batch=4, inflight=2, rr=(0, 1), depth=1 << 12, tcache=None):
    inl = tile.Link(depth, 1232)
    outl = tile.Link(depth, tile.TPU_DCACHE_MTU)
    vt = tile.VerifyTile(inl, outl, verifier, hashmap_seed=seed, batch_txn_max=batch, inflight_max=inflight,
                         round_robin_idx=rr[0], round_robin_cnt=rr[1], log_max=1 << 16)
    for p in payloads:
        inl.publish(p)
    vt.run(len(payloads), timeout_s=30)
    return vt, inl, outl


def test_verify_tile_reference_sequences(fixtures, oracle):
    """test_verify.c:159-317 sequences through the tile: SUCCESS / DEDUP /
    FAILED exactly as the reference's fd_txn_verify returns them, with the
    duplicates inside one batch and across batches."""
    v1, v2 = fixtures["test_verify.valid_txn_1sig"], fixtures["test_verify.valid_txn_2sigs"]
    i2, same1 = fixtures["test_verify.invalid_txn_2sigs"], fixtures["test_verify.invalid_txn_same_1sig"]
    same64 = fixtures["test_verify.invalid_txn_1sig_same_64bit"]
    S, F, D = tile.VERIFY_SUCCESS, tile.VERIFY_FAILED, tile.VERIFY_DEDUP
    for batch in (1, 3, 16):
        ver = tile.PyVerifier(oracle_fn(oracle), slots=2, lag=1)
        seq = [v2, v2, v2, v1, v1, v1]
        vt, _, outl = _run_tile(seq, ver, batch=batch)
        assert vt.log()[1].tolist() == [S, D, D, S, D, D]
        assert len(outl.drain()) == 2
        vt, _, _ = _run_tile([i2, i2], tile.PyVerifier(oracle_fn(oracle)), batch=batch)
        assert vt.log()[1].tolist() == [F, F]                  # no dedup for failed txns
        vt, _, _ = _run_tile([same1, v1], tile.PyVerifier(oracle_fn(oracle)), batch=batch)
        assert vt.log()[1].tolist() == [F, S]                  # front-running invalid txn is not cached
        vt, _, _ = _run_tile([v1, same1], tile.PyVerifier(oracle_fn(oracle)), batch=batch)
        assert vt.log()[1].tolist() == [S, D]                  # ...but is deduped after the valid one
        vt, _, _ = _run_tile([v1, same64], tile.PyVerifier(oracle_fn(oracle)), batch=batch)
        assert vt.log()[1].tolist() == [S, F]                  # same low 64 bits is not a dup


def test_verify_tile_tcache_reset(fixtures, oracle):
    """test_verify.c:264-277: clearing the tcache between phases."""
    v1, same1 = fixtures["test_verify.valid_txn_1sig"], fixtures["test_verify.invalid_txn_same_1sig"]
    inl, outl = tile.Link(64, 1232), tile.Link(64, tile.TPU_DCACHE_MTU)
    vt = tile.VerifyTile(inl, outl, tile.PyVerifier(oracle_fn(oracle)), batch_txn_max=8, log_max=64)
    inl.publish(same1); inl.publish(v1)
    vt.run(2)
    vt.tcache.reset()
    inl.publish(v1); inl.publish(same1)
    vt.run(4)
    assert vt.log()[1].tolist() == [-1, 0, 0, -2]


def test_verify_tile_output_format(oracle, quic_corpus):
    """Published frags are [payload][pad to 2][fd_txn_t][u16 payload_sz]
    with sig = fd_hash(seed, sig0, 64) and ctl 0 (fd_verify.c:93-147)."""
    arena, txns, _ = quic_corpus
    ps = [bytes(arena[int(t["sig_off"]) - 1: int(t["msg_off"]) + int(t["msg_sz"])]) for t in txns[:300]]
    seed = 0x1234
    vt, _, outl = _run_tile(ps, tile.PyVerifier(oracle_fn(oracle)), seed=seed, batch=64)
    outs = outl.drain()
    _, exp = tile_model.verify_tile_model(ps, seed, oracle_fn(oracle))
    assert len(outs) == len(exp) == vt.stats()["published"]
    for (meta, frag), (p, raw, tag) in zip(outs, exp):
        assert meta["sig"] == tag and meta["ctl"] == 0
        toff = (len(p) + 1) & ~1
        assert meta["sz"] == toff + len(raw) + 2
        pay, traw = tile.split_verify_output(frag)
        assert pay == p and traw == raw


def _mixed_stream(n, seed, oracle_ok=True):
    """Generated single- and multi-signature txns (10% corrupted) with
    duplicates re-sent at short and long distances (inside and beyond the
    16-deep tcache) and some unparseable frags."""
    rnd = random.Random(seed)
    junk = random.Random(seed ^ 0x7A7A)
    a1, t1, _ = workload.cfg1(n // 2, seed=seed)
    a3, t3, _ = workload.cfg3(n // 4, seed=seed + 1)
    base = workload.payloads(a1, t1) + workload.payloads(a3, t3)
    rnd.shuffle(base)
    out = []
    for p in base:
        out.append(p)
        r = rnd.random()
        if r < 0.15 and out:
            out.append(out[-1 - min(int(rnd.expovariate(1 / 12)), len(out) - 1)])
        elif r < 0.18:
            out.append(p[:-3])                                  # truncated: parse failure
        elif r < 0.20:
            q = bytearray(p); q[0] = 0; out.append(bytes(q))     # zero signatures
        elif r < 0.21:                                           # random bytes behind a plausible count
            out.append(bytes([junk.randrange(1, 13)]) +
                       bytes(junk.getrandbits(8) for _ in range(junk.randrange(64, 1232))))
    return out


@pytest.mark.parametrize("batch,inflight,lag,rr", [(1, 1, 0, (0, 1)), (7, 2, 2, (0, 1)), (64, 3, 1, (1, 3)),
                                                    (1000, 2, 0, (0, 1))])
def test_verify_tile_vs_sequential_model(oracle, batch, inflight, lag, rr):
    """The batched, pipelined tile produces the reference loop's outcome for
    every frag and the same published stream, for any batch size / number
    of batches in flight / verifier latency / round-robin share."""
    ps = _mixed_stream(800, seed=batch * 31 + lag)
    seed = 0x77 + batch
    ver = tile.PyVerifier(oracle_fn(oracle), slots=inflight, lag=lag)
    vt, _, outl = _run_tile(ps, ver, seed=seed, batch=batch, inflight=inflight, rr=rr)
    exp_out, exp_pub = tile_model.verify_tile_model(ps, seed, oracle_fn(oracle), rr_idx=rr[0], rr_cnt=rr[1])
    seqs, codes = vt.log()
    assert seqs.tolist() == list(range(len(ps)))
    assert codes.tolist() == exp_out
    outs = outl.drain()
    assert [(m["sig"], tile.split_verify_output(f)[0]) for m, f in outs] == [(t, p) for p, _, t in exp_pub]
    st = vt.stats()
    assert st["published"] == exp_out.count(0) and st["dedup"] == exp_out.count(-2)
    assert st["verify_failed"] == exp_out.count(-1) and st["parse_fail"] == exp_out.count(1)
    assert st["filtered_rr"] == exp_out.count(2) and st["overrun"] == 0
    assert exp_out.count(-2) > 10 and exp_out.count(-1) > 10 and exp_out.count(1) > 5


def test_verify_tile_signature_cap(oracle):
    """Batches close before their signature count can exceed batch_sig_max
    (the engines' max_sig), so a stream of 12-signature transactions never
    builds a batch the engine rejects; outcomes still match the model."""
    a3, t3, _ = workload.make_txns(120, seed=0xCA9, multi=True, max_sigs=12)
    ps = workload.payloads(a3, t3)
    cap = 40
    seen = []

    def fn(arena, txns):
        cnt = txns["sig_cnt"].astype(np.int64)
        seen.append(int(np.where((cnt >= 1) & (cnt <= 16), cnt, 0).sum()))
        return oracle_fn(oracle)(arena, txns)

    inl, outl = tile.Link(1 << 10, 1232), tile.Link(1 << 10, tile.TPU_DCACHE_MTU)
    vt = tile.VerifyTile(inl, outl, tile.PyVerifier(fn), batch_txn_max=64, batch_sig_max=cap, log_max=1 << 12)
    for q in ps:
        inl.publish(q)
    vt.run(len(ps), timeout_s=30)
    assert max(seen) <= cap and sum(seen) == int(t3["sig_cnt"].sum())
    exp_out, _ = tile_model.verify_tile_model(ps, 0x5EEDF00D, oracle_fn(oracle))
    assert vt.log()[1].tolist() == exp_out


def test_verify_tile_recovers_from_rejected_batch(oracle, fixtures):
    """A batch the verifier rejects as malformed (FDGPU_ERR_INVAL) fails its
    transactions (verify_errors, nothing published) and the tile keeps
    running: the next batches verify normally."""
    v1, v2 = fixtures["test_verify.valid_txn_1sig"], fixtures["test_verify.valid_txn_2sigs"]
    state = {"n": 0}
    inner = tile.PyVerifier(oracle_fn(oracle))

    def fn(arena, txns):
        return oracle_fn(oracle)(arena, txns)

    ver = tile.PyVerifier(fn)
    orig_submit = ver._submit

    def submit(ctx, arena, arena_sz, txns, n):
        state["n"] += 1
        if state["n"] == 1:
            return -10                                            # FDGPU_ERR_INVAL
        return orig_submit(ctx, arena, arena_sz, txns, n)

    ver._submit = tile.SUBMIT_FN(submit)
    ver.struct = tile.Verifier(None, ver._submit, ver._poll)
    inl, outl = tile.Link(64, 1232), tile.Link(64, tile.TPU_DCACHE_MTU)
    vt = tile.VerifyTile(inl, outl, ver, batch_txn_max=2, log_max=64)
    for q in (v1, v2, v1, v2):
        inl.publish(q)
    vt.run(4, timeout_s=10)
    st = vt.stats()
    F, S, D = tile.VERIFY_FAILED, tile.VERIFY_SUCCESS, tile.VERIFY_DEDUP
    assert vt.log()[1].tolist() == [F, F, S, S]                   # first batch rejected, tcache untouched
    assert st["verify_errors"] == 2 and st["published"] == 2
    del inner


def test_verify_tile_out_flow_control(oracle):
    """With a reliable consumer (out fseq), the tile never runs more than
    out_depth frags ahead of it and resumes when it advances."""
    ps = _mixed_stream(200, seed=5)
    inl, outl = tile.Link(1 << 10, 1232), tile.Link(16, tile.TPU_DCACHE_MTU)
    vt = tile.VerifyTile(inl, outl, tile.PyVerifier(oracle_fn(oracle)), batch_txn_max=32, flow_control=True)
    for p in ps:
        inl.publish(p)
    _, exp_pub = tile_model.verify_tile_model(ps, 0x5EEDF00D, oracle_fn(oracle))
    got = []
    for _ in range(200000):
        vt.step()
        rc, meta, _ = outl.poll(int(outl.fseq[0]))            # slow consumer: one frag per step
        if rc == 1:
            got.append(meta["sig"])
            outl.fseq[0] += 1
        assert vt.stats()["published"] - int(outl.fseq[0]) <= 16
        if len(got) == len(exp_pub):
            break
    vt.flush()
    assert got == [t for _, _, t in exp_pub]
    assert vt.stats()["backpressure"] > 0


def test_verify_tile_overrun_accounting(oracle):
    """A producer lapping the tile (quic->verify has no backpressure): lost
    frags are counted, never half-read; every frag the tile did take is
    resolved like the model."""
    ps = _mixed_stream(400, seed=9)
    inl, outl = tile.Link(64, 1232), tile.Link(1 << 12, tile.TPU_DCACHE_MTU)
    vt = tile.VerifyTile(inl, outl, tile.PyVerifier(oracle_fn(oracle)), batch_txn_max=16, log_max=1 << 12)
    for p in ps[:40]:
        inl.publish(p)
    vt.step()
    for p in ps[40:]:                                          # laps the 64-deep mcache
        inl.publish(p)
    vt.run(len(ps), timeout_s=30)
    st = vt.stats()
    seqs, codes = vt.log()
    assert st["overrun"] > 0 and len(seqs) == len(ps)
    assert (codes == tile.LOG_LOST).sum() == st["overrun"]


# ------------------------------------------------------------ dedup tile

def test_dedup_tile_two_verify_tiles(oracle):
    """Two verify tiles (round robin 0/2 and 1/2) -> one dedup tile with a
    large tcache: output is every verified txn once, in service order, with
    sig 0 (fd_dedup.c:194-205)."""
    ps = _mixed_stream(600, seed=21)
    inl = tile.Link(1 << 11, 1232)
    outs = [tile.Link(1 << 11, tile.TPU_DCACHE_MTU) for _ in range(2)]
    vts = [tile.VerifyTile(inl, outs[k], tile.PyVerifier(oracle_fn(oracle)), hashmap_seed=100 + k,
                           batch_txn_max=50, round_robin_idx=k, round_robin_cnt=2) for k in range(2)]
    for p in ps:
        inl.publish(p)
    for vt in vts:
        vt.run(len(ps), timeout_s=30)
    dout = tile.Link(1 << 11, tile.TPU_DCACHE_MTU)
    dt = tile.DedupTile(outs, dout, hashmap_seed=0xD5, tcache_depth=1 << 16)
    dt.run_until_idle()
    # dedup services its in links round robin, one frag each per pass
    streams = [[f for _, f in o.drain()] for o in outs]
    order, idx, k = [], [0, 0], 0
    while idx[0] < len(streams[0]) or idx[1] < len(streams[1]):
        for j in (k % 2, (k + 1) % 2):
            if idx[j] < len(streams[j]):
                order.append(streams[j][idx[j]]); idx[j] += 1
        k += 1
    exp = tile_model.dedup_model(order, 0xD5, 1 << 16)
    got = dout.drain()
    assert [f for _, f in got] == exp
    assert all(m["sig"] == 0 for m, _ in got)
    st = dt.stats()
    assert st["in_frags"] == len(order) and st["published"] == len(exp) and st["dup"] == len(order) - len(exp)
    # across the two verify tiles, cross-tile duplicates only dedup here
    assert st["dup"] > 0


def test_dedup_tile_reliable_links_publish_progress(oracle):
    """reliable=True (the verify -> dedup links of fd_topo): the dedup tile
    stores its next seq of each in link into that link's fseq as it consumes
    -- what a flow-controlled verify tile takes its credits from -- and a
    tile without it leaves the fseqs alone."""
    ps = _mixed_stream(300, seed=22)
    inl = tile.Link(1 << 10, 1232)
    outs = [tile.Link(1 << 10, tile.TPU_DCACHE_MTU) for _ in range(2)]
    vts = [tile.VerifyTile(inl, outs[k], tile.PyVerifier(oracle_fn(oracle)), hashmap_seed=100 + k,
                           batch_txn_max=50, round_robin_idx=k, round_robin_cnt=2) for k in range(2)]
    for p in ps:
        inl.publish(p)
    for vt in vts:
        vt.run(len(ps), timeout_s=30)
    pub = [int(vt.stats()["published"]) for vt in vts]
    f0 = [int(o.fseq[0]) for o in outs]
    unrel = tile.DedupTile(outs, tile.Link(1 << 10, tile.TPU_DCACHE_MTU), tcache_depth=1 << 12)
    unrel.run_until_idle()
    assert [int(o.fseq[0]) for o in outs] == f0
    rel = tile.DedupTile(outs, tile.Link(1 << 10, tile.TPU_DCACHE_MTU), tcache_depth=1 << 12, reliable=True)
    assert rel.run_until_idle() == sum(pub)
    assert [int(o.fseq[0]) for o in outs] == [o.seq0 + n for o, n in zip(outs, pub)]


def _verify_outputs(ps):
    """verify-tile out frags ([payload][pad][fd_txn_t][u16 payload sz]) of the parseable payloads"""
    outs = []
    for p in ps:
        sz, raw = tile.txn_parse(p)
        if sz:
            outs.append(p + (b"\0" if len(p) & 1 else b"") + raw + len(p).to_bytes(2, "little"))
    return outs


def test_dedup_tile_steady_state_tcache_vs_model():
    """The dedup tile with its tcache in the steady state (filled with
    `depth` other tags first: every insert evicts) against the model fed the
    same tags: same published stream, same dups -- the eviction order, the
    prefetched map lines and the huge-page region change nothing -- over a
    link that also carries frags whose trailers lie (sizes and offsets out of
    range: counted corrupt, never read past the frag)."""
    rng = np.random.default_rng(0xDEDE)
    base = _verify_outputs(_mixed_stream(700, seed=23))
    stream = []
    for k in range(3000):
        r = rng.random()
        if r < 0.08:                                  # a frag whose trailer lies
            f = bytearray(rng.integers(0, 256, size=int(rng.integers(2, 300)), dtype=np.uint8).tobytes())
            f[-2:] = int(rng.integers(0, 65536)).to_bytes(2, "little")
            stream.append(bytes(f))
        else:                                         # a verified txn, often seen before (near or far back)
            stream.append(base[int(rng.integers(0, len(base)))])
    depth = 1024
    inl = tile.Link(1 << 12, tile.TPU_DCACHE_MTU)
    for f in stream:
        inl.publish(f)
    dout = tile.Link(1 << 12, tile.TPU_DCACHE_MTU)
    dt = tile.DedupTile([inl], dout, hashmap_seed=0xD5, tcache_depth=depth)
    assert dt.tcache_fill(depth + 77, seed=5) == 0
    dt.run_until_idle()
    model = tile_model.TCacheModel(depth)
    for t in np.random.default_rng(5).integers(1, 2 ** 63, size=depth + 77, dtype=np.uint64):
        model.insert(int(t))
    exp, corrupt = [], 0
    for f in stream:
        psz = int.from_bytes(f[-2:], "little")
        toff = (psz + 1) & ~1
        if toff + ctypes.sizeof(tile.TxnHdr) + 2 > len(f):
            corrupt += 1
            continue
        so = tile.TxnHdr.from_buffer_copy(f[toff:toff + ctypes.sizeof(tile.TxnHdr)]).signature_off
        if so + 64 > len(f):
            corrupt += 1
            continue
        if not model.insert(tile.fd_hash(0xD5, f[so:so + 64])):
            exp.append(f)
    st = dt.stats()
    assert [f for _, f in dout.drain()] == exp
    assert st["published"] == len(exp) and st["corrupt"] == corrupt and corrupt > 100
    assert st["in_frags"] == len(stream) and st["dup"] == len(stream) - len(exp) - corrupt


def test_dedup_tile_reference_depth():
    """At the reference's signature_cache_size (4,194,302, default.toml:910),
    the tile's default: a txn seen again after 18 K other frags is dropped,
    where a 16,384-deep tcache has forgotten it and publishes it again."""
    def sig0(f):
        so = tile.TxnHdr.from_buffer_copy(tile.split_verify_output(f)[1]).signature_off
        return so, f[so:so + 64]
    outs = list({sig0(f)[1]: f for f in _verify_outputs(_mixed_stream(500, seed=24))}.values())

    def variant(f, c):                              # the same frag with another first signature
        so = sig0(f)[0]
        b = bytearray(f)
        b[so:so + 3] = bytes((0xA5, c >> 8, c & 0xFF))
        return bytes(b)
    filler = [variant(f, c) for c in range((1 << 14) // len(outs) + 2) for f in outs]
    stream = outs + filler + outs                   # the second copies ~18 K frags after the first
    assert len({sig0(f)[1] for f in stream}) == len(outs) + len(filler) > (1 << 14) + len(outs)
    for depth, exp in ((4194302, len(outs) + len(filler)), (1 << 14, len(stream))):
        inl = tile.Link(1 << 16, tile.TPU_DCACHE_MTU)
        for f in stream:
            inl.publish(f)
        dout = tile.Link(1 << 10, tile.TPU_DCACHE_MTU)
        dt = tile.DedupTile([inl], dout, tcache_depth=depth)
        assert dt.run_until_idle() == len(stream)
        st = dt.stats()
        assert st["published"] == exp and st["dup"] == len(stream) - exp, (depth, st)


def test_dedup_tile_unparsed_link(oracle, fixtures):
    """A gossip-style link of raw txns is parsed by the dedup tile itself
    (fd_dedup.c:147-192) and produces the verify tile's trailer format."""
    raw_l = tile.Link(64, tile.TPU_DCACHE_MTU)
    ver_l = tile.Link(64, tile.TPU_DCACHE_MTU)
    dout = tile.Link(64, tile.TPU_DCACHE_MTU)
    v1 = fixtures["test_verify.valid_txn_1sig"]
    raw_l.publish(v1)
    raw_l.publish(b"\x01garbage")
    dt = tile.DedupTile([raw_l, ver_l], dout, tcache_depth=1024, unparsed_in_cnt=1)
    dt.run_until_idle()
    got = dout.drain()
    assert len(got) == 1
    pay, traw = tile.split_verify_output(got[0][1])
    assert pay == v1 and traw == tile.txn_parse(v1)[1]
    assert dt.stats()["parse_fail"] == 1


# -------------------------------------------------------------- producer

def test_producer_thread_feeds_tile(oracle):
    """The line-rate producer thread publishes into a deep link while the
    tile consumes it concurrently; everything is resolved exactly once."""
    ps = _mixed_stream(400, seed=33)
    arena, offs, sizes = workload.pack_payloads(ps)
    inl, outl = tile.Link(1 << 10, 1232), tile.Link(1 << 10, tile.TPU_DCACHE_MTU)
    vt = tile.VerifyTile(inl, outl, tile.PyVerifier(oracle_fn(oracle)), batch_txn_max=32, log_max=1 << 12)
    prod = tile.Producer(inl, arena, offs, sizes, rate_tps=200000)
    vt.run(len(ps), timeout_s=60)
    n, el = prod.join()
    assert n == len(ps) and el > 0
    exp, _ = tile_model.verify_tile_model(ps, 0x5EEDF00D, oracle_fn(oracle))
    assert vt.log()[1].tolist() == exp


def test_tile_header_exports():
    """libfd_verify_tile.so exports every function include/fd_verify_tile.h declares."""
    L = tile.lib()
    names = tile.header_functions()
    assert len(names) > 30
    for n in names:
        assert hasattr(L, n), n


def test_txn_peek_agrees_with_parse(quic_corpus, fixtures):
    """fdt_txn_peek (the trailer reservation of the GPU-parse verify tile)
    returns fd_txn_parse's footprint and the signature count for every
    payload that parses -- the QUIC corpus, the fixtures (legacy and v0 with
    lookup tables), generated txns, single-byte mutations and truncations of
    the fixtures, random splices -- and never reads past the payload (run
    under ASan/UBSan by test_sanitize.py)."""
    rnd = random.Random(0x9EE)
    arena, txns, _ = quic_corpus
    cases = [bytes(arena[int(t["sig_off"]) - 1: int(t["msg_off"]) + int(t["msg_sz"])]) for t in txns[:1000]]
    base = list(fixtures.values())
    cases += base
    for cfgf in (workload.cfg1, workload.cfg3):
        a, tx, _ = cfgf(300, seed=12)
        cases += workload.payloads(a, tx)
    for p in base:
        cases += [p[:n] for n in range(len(p) + 1)]
        for _ in range(400):
            q = bytearray(p)
            q[rnd.randrange(len(q))] = rnd.getrandbits(8)
            cases.append(bytes(q))
    for _ in range(1000):
        a, b = rnd.choice(base), rnd.choice(base)
        cases.append(a[:rnd.randrange(len(a) + 1)] + b[rnd.randrange(len(b) + 1):])
    parsed = 0
    for p in cases:
        fp, raw = tile.txn_parse(p)
        pk, sc = tile.txn_peek(p)
        if fp:
            parsed += 1
            d = tile.txn_decode(raw)
            assert pk == fp and sc == d["signature_cnt"] and d["signature_off"] == 1, p.hex()[:80]
        assert pk <= tile.TXN_MAX_SZ
    for _ in range(20000):                                       # random bytes: reservations stay bounded
        p = bytes([rnd.randrange(1, 13)]) + bytes(rnd.getrandbits(8) for _ in range(rnd.randrange(0, 1232)))
        assert tile.txn_peek(p)[0] <= tile.TXN_MAX_SZ
    assert parsed > 2000


def test_tagring_equals_tcache():
    """fdt_tagring (the verify tile's 16-deep tcache as a ring scan) answers
    every query and insert exactly as fdt_tcache of the same depth (the
    reference's FD_TCACHE_QUERY / FD_TCACHE_INSERT, fd_tcache.h:281-404), on
    streams with repeats at every distance and the null tag."""
    import ctypes
    L = tile.lib()
    rnd = random.Random(0x7A6)
    for depth in (1, 2, 5, 16, 32):
        tc = tile.TCache(depth, 64 if depth <= 16 else 128)
        ring = ctypes.create_string_buffer(8 * (32 + 2))
        L.fdt_tagring_init(ring, depth)
        pool = [rnd.getrandbits(64) for _ in range(3 * depth + 4)] + [0]
        for _ in range(30000):
            tag = rnd.choice(pool) if rnd.random() < 0.8 else rnd.getrandbits(64)
            if rnd.random() < 0.5:
                assert L.fdt_tagring_query(ring, tag) == tc.query(tag), (depth, tag)
            else:
                assert L.fdt_tagring_insert(ring, tag) == tc.insert(tag), (depth, tag)
