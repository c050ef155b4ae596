"""TPU stream reassembly (the quic -> verify link's producer,
src/disco/quic/fd_tpu.h:20-246) and the verify tile reading from its slot
arena with the reasm chunk bounds (fd_verify.c:186-191).  Slot ownership,
eviction and append rules are the ones fd_tpu.h documents; the tile's
outcomes are checked against the sequential model of the reference loop."""
import random

import pytest

from firedancer_amd import tile
import tile_model
from test_tile import _mixed_stream


def _states(r):
    return [r.state(i) for i in range(r.depth + r.burst)]


def test_reasm_slot_accounting():
    """Exactly depth slots published and burst owned by reassembly, always."""
    r = tile.TpuReasm(8, 4)
    rnd = random.Random(1)
    busy = []
    for step in range(500):
        op = rnd.random()
        if op < 0.4 or not busy:
            busy.append(r.prepare())
            busy = [s for s in dict.fromkeys(busy) if r.state(s) == tile.REASM_BUSY]   # evicted + re-prepared
        elif op < 0.8:
            s = busy.pop(rnd.randrange(len(busy)))
            assert r.append(s, b"x" * rnd.randrange(1, 100), 0) == tile.REASM_SUCCESS
            assert r.publish(s) == tile.REASM_SUCCESS
        else:
            r.cancel(busy.pop(rnd.randrange(len(busy))))
        st = _states(r)
        assert st.count(tile.REASM_PUB) == 8
        assert st.count(tile.REASM_FREE) + st.count(tile.REASM_BUSY) == 4


def test_reasm_fifo_eviction():
    """With every slot busy, prepare cancels the least recently prepared
    stream (fd_tpu.h: "cancelling the least recently prepared reassembly")."""
    r = tile.TpuReasm(4, 3)
    a, b, c_ = r.prepare(), r.prepare(), r.prepare()
    assert len({a, b, c_}) == 3
    d = r.prepare()
    assert d == a and r.state(b) == r.state(c_) == tile.REASM_BUSY
    assert r.append(b, b"abc", 0) == tile.REASM_SUCCESS
    e = r.prepare()                     # b was prepared before c_: b goes next
    assert e == b and r.state(c_) == tile.REASM_BUSY


def test_reasm_append_rules():
    r = tile.TpuReasm(4, 2)
    s = r.prepare()
    assert r.append(s, b"0123456789", 0) == tile.REASM_SUCCESS
    assert r.append(s, b"56789abc", 5) == tile.REASM_SUCCESS          # overlap: seen prefix skipped
    assert r.append(s, b"12", 1) == tile.REASM_SUCCESS                 # fully seen: no-op
    assert r.publish(s) == tile.REASM_SUCCESS
    rc, meta, _ = r.poll(0)
    assert rc == 1 and r.payload(meta) == b"0123456789abc"
    assert meta["chunk"] >= r.chunk0 and meta["chunk"] <= r.wmark
    assert r.publish(s) == tile.REASM_ERR_STATE                        # already published
    g = r.prepare()
    assert r.append(g, b"zz", 3) == tile.REASM_ERR_SKIP and r.state(g) == tile.REASM_FREE
    h = r.prepare()
    assert r.append(h, b"q" * 1232, 0) == tile.REASM_SUCCESS
    assert r.append(h, b"q", 1232) == tile.REASM_ERR_SZ and r.state(h) == tile.REASM_FREE
    assert r.append(h, b"q", 0) == tile.REASM_ERR_STATE


def test_reasm_payload_stable_for_depth_publishes():
    """A published payload is not overwritten until `depth` later publishes
    (the slot stays mcache-owned), and is reused right after."""
    r = tile.TpuReasm(4, 2)
    msgs = [bytes([i]) * (50 + i) for i in range(12)]
    chunks = []
    for i, m in enumerate(msgs):
        s = r.prepare()
        r.append(s, m, 0)
        r.publish(s)
        chunks.append(r.poll(i)[1]["chunk"])
        for j in range(max(0, i - 3), i + 1):                          # the last depth frags intact
            rc, meta, _ = r.poll(j)
            assert rc == 1 and r.payload(meta) == msgs[j]
    assert r.poll(0)[0] == -1                                          # line reused: overrun


def _reasm_tile_run(oracle, depth, burst, batch, verifier, n=600):
    """QUIC-style fragmented streams (interleaved, in-order pieces with
    repeats) reassembled and published, the verify tile consuming the slot
    arena concurrently: every frag's outcome and the published stream match
    the reference loop's model over the publish order."""
    ps = [p for p in _mixed_stream(n, seed=depth + burst) if len(p) <= 1232]
    rnd = random.Random(depth)
    r = tile.TpuReasm(depth, burst)
    outl = tile.Link(1 << 13, tile.TPU_DCACHE_MTU)          # holds every output (drained at the end)
    vt = tile.VerifyTile(r, outl, verifier, batch_txn_max=batch, log_max=1 << 14)
    i, open_, pub_order = 0, [], []                  # open_: streams in progress [slot, payload, sent]
    while i < len(ps) or open_:
        if i < len(ps) and len(open_) < burst and (not open_ or rnd.random() < 0.5):
            open_.append([r.prepare(), ps[i], 0])
            i += 1
            continue
        k = rnd.randrange(len(open_))
        slot, p, sent = open_[k]
        n = rnd.randrange(1, 400)
        back = rnd.randrange(0, min(sent, 20) + 1)                    # resend a little
        assert r.append(slot, p[sent - back:sent + n], sent - back) == tile.REASM_SUCCESS
        open_[k][2] = min(len(p), sent + n)
        if open_[k][2] == len(p):
            assert r.publish(slot) == tile.REASM_SUCCESS
            pub_order.append(p)
            open_.pop(k)
            vt.step()
    vt.run(r.next_seq, timeout_s=30)
    seqs, codes = vt.log()
    assert len(seqs) == len(ps) == r.next_seq and vt.stats()["overrun"] == 0
    exp_out, exp_pub = tile_model.verify_tile_model(pub_order, 0x5EEDF00D, lambda a, t: oracle.verify_txns(a, t))
    assert codes.tolist() == exp_out
    assert [tile.split_verify_output(f)[0] for _, f in outl.drain()] == [p for p, _, _ in exp_pub]
    assert exp_out.count(0) > 100 and exp_out.count(-1) > 10


@pytest.mark.parametrize("depth,burst,batch", [(1 << 10, 16, 32), (64, 4, 8)])
def test_verify_tile_reads_reasm_link(oracle, depth, burst, batch):
    _reasm_tile_run(oracle, depth, burst, batch, tile.PyVerifier(lambda a, t: oracle.verify_txns(a, t)))


@pytest.mark.gpu
def test_verify_tile_reads_reasm_link_gpu(oracle, engine):
    ver = tile.EngineVerifier([engine])
    try:
        _reasm_tile_run(oracle, 1 << 12, 32, 256, ver, n=4000)
    finally:
        ver.close()
