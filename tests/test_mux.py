"""The reference's mux callback API restated (fdt_mux_run / fdt_mux_publish,
src/disco/mux/fd_mux.h:106-299, fd_mux.c:387-699) and the verify tile written
against it (fdgpu_vmux: fd_verify.c:232-246 with FD_MUX_FLAG_COPY |
FD_MUX_FLAG_MANUAL_PUBLISH), on CPU.  The tile's verifier here is a
PyVerifier over the CPU oracle; tests/test_tile_gpu.py runs the same tile
over the MI355X engines."""
import ctypes as c
import random
import threading
import time

import numpy as np
import pytest

from firedancer_amd import tile, workload
import tile_model
from test_tile import _mixed_stream, oracle_fn

u64 = c.c_uint64
BEFORE_CREDIT = c.CFUNCTYPE(None, c.c_void_p, c.c_void_p)
AFTER_CREDIT = c.CFUNCTYPE(None, c.c_void_p, c.c_void_p, c.POINTER(c.c_int))
BEFORE_FRAG = c.CFUNCTYPE(None, c.c_void_p, u64, u64, u64, c.POINTER(c.c_int))
DURING_FRAG = c.CFUNCTYPE(None, c.c_void_p, u64, u64, u64, u64, u64, c.POINTER(c.c_int))
AFTER_FRAG = c.CFUNCTYPE(None, c.c_void_p, u64, u64, c.POINTER(u64), c.POINTER(u64), c.POINTER(u64),
                         c.POINTER(u64), c.POINTER(c.c_int), c.c_void_p)
HOUSEKEEPING = c.CFUNCTYPE(None, c.c_void_p)


def _mux_cfg(in_links, out_link=None, flags=tile.MUX_FLAG_DEFAULT, out_fseq=None, cr_max=0):
    mc = tile.MuxCfg()
    mc.in_cnt = len(in_links)
    for i, ln in enumerate(in_links):
        mc.in_mcache[i], mc.in_depth[i], mc.in_seq0[i] = ln.mcache_ptr, ln.depth, ln.seq0
    if out_link is not None:
        mc.out_mcache, mc.out_depth, mc.out_seq0 = out_link.mcache_ptr, out_link.depth, out_link.seq0
    if out_fseq is not None:
        mc.out_cnt, mc.out_fseq[0] = 1, out_fseq.ctypes.data
    mc.flags, mc.burst, mc.cr_max, mc.lazy_iters = flags, 1, cr_max, 4
    return mc


class MuxThread:
    def __init__(self, cfg, cb, ctx=None):
        self.cfg, self.cb, self.ctx = cfg, cb, ctx
        self.halt, self.stats, self.rc = u64(0), tile.MuxStats(), None
        self.th = threading.Thread(target=self._body, daemon=True)
        self.th.start()

    def _body(self):
        self.rc = tile.lib().fdt_mux_run(c.byref(self.cfg), c.byref(self.cb), self.ctx, c.byref(self.halt),
                                         c.byref(self.stats))

    def stop(self):
        self.halt.value = 1
        self.th.join(30)
        assert not self.th.is_alive()
        return self.rc


def _wait(cond, timeout=30.0):
    t0 = time.time()
    while not cond():
        assert time.time() - t0 < timeout, "timed out"
        time.sleep(0.001)


def test_mux_relays_frags_without_callbacks():
    """No callbacks, default flags: every in frag is republished on the out
    mcache with its sig / chunk / sz / ctl / tsorig (the zero-copy mux), and
    two ins are serviced round robin, each in order."""
    a, b = tile.Link(64, 1232), tile.Link(64, 1232)
    out = tile.Link(256, 1232)
    for i in range(40):
        a.publish(bytes([i]) * (10 + i), sig=1000 + i)
        b.publish(bytes([i]) * 5, sig=2000 + i)
    m = MuxThread(_mux_cfg([a, b], out), tile.MuxCallbacks())
    _wait(lambda: out.poll(out.seq0 + 79)[0] == 1)
    assert m.stop() == 0
    got = out.drain()
    assert len(got) == 80 and m.stats.published == 80
    sa = [mt["sig"] for mt, _ in got if mt["sig"] < 2000]
    sb = [mt["sig"] for mt, _ in got if mt["sig"] >= 2000]
    assert sa == list(range(1000, 1040)) and sb == list(range(2000, 2040))
    for mt, _ in got:                                      # chunk / sz point at the in link's payload
        src = a if mt["sig"] < 2000 else b
        i = mt["sig"] % 1000
        assert bytes(src.dcache[mt["chunk"] * 64: mt["chunk"] * 64 + mt["sz"]]) == \
            (bytes([i]) * (10 + i) if src is a else bytes([i]) * 5)


def test_mux_callback_order_and_filters():
    """before_frag sees (seq, sig) and can drop a frag unread; during_frag
    sees chunk/sz and can filter; after_frag runs only for unfiltered frags
    and can rewrite sig/sz before the mux publishes; after_credit runs every
    loop with poll_in defaulting to 1 (fd_mux.c:559-660)."""
    inl = tile.Link(128, 1232)
    out = tile.Link(128, 1232)
    for i in range(60):
        inl.publish(bytes([i & 255]) * 20, sig=i * 7)
    ev = {"before": [], "during": [], "after": [], "credit": 0}

    def before(ctx, idx, seq, sig, filt):
        ev["before"].append((seq, sig))
        if seq % 2:
            filt[0] = 1

    def during(ctx, idx, seq, sig, chunk, sz, filt):
        ev["during"].append(seq)
        assert sz == 20
        if seq % 3 == 0:
            filt[0] = 1

    def after(ctx, idx, seq, opt_sig, opt_chunk, opt_sz, opt_tsorig, filt, mux):
        ev["after"].append(seq)
        opt_sig[0] = 100000 + seq
        opt_sz[0] = 8

    def credit(ctx, mux, poll_in):
        ev["credit"] += 1
        assert poll_in[0] == 1

    fns = [BEFORE_FRAG(before), DURING_FRAG(during), AFTER_FRAG(after), AFTER_CREDIT(credit)]
    cb = tile.MuxCallbacks()
    cb.before_frag, cb.during_frag, cb.after_frag, cb.after_credit = [c.cast(f, c.c_void_p) for f in fns]
    m = MuxThread(_mux_cfg([inl], out), cb)
    exp = [s for s in range(60) if s % 2 == 0 and s % 3]
    _wait(lambda: len(ev["before"]) >= 60)
    assert m.stop() == 0
    assert [s for s, _ in ev["before"]][:60] == list(range(60))
    assert all(sig == 7 * s for s, sig in ev["before"])
    assert ev["during"] == [s for s in range(60) if s % 2 == 0]
    assert ev["after"] == exp
    got = out.drain()
    assert [mt["sig"] for mt, _ in got] == [100000 + s for s in exp] and all(mt["sz"] == 8 for mt, _ in got)
    assert ev["credit"] >= 60
    st = m.stats.as_dict()
    assert st["filtered_before"] == 30 and st["filtered_after"] == 10 and st["published"] == len(exp)


def test_mux_credits_backpressure():
    """With one reliable consumer whose fseq does not move, the mux exposes at
    most cr_max frags, then spins backpressured (after_credit not called)
    until the consumer's fseq advances (fd_mux.c:467-487,548-556)."""
    inl = tile.Link(64, 1232)
    out = tile.Link(64, 1232)
    for i in range(20):
        inl.publish(b"x" * 10, sig=i)
    fseq = np.zeros(1, dtype=np.uint64)
    m = MuxThread(_mux_cfg([inl], out, out_fseq=fseq, cr_max=4), tile.MuxCallbacks())
    _wait(lambda: out.poll(3)[0] == 1)
    time.sleep(0.05)
    assert out.poll(4)[0] == 0                             # 4 exposed, no credit for a 5th
    fseq[0] = 3                                            # consumer read 3 frags
    _wait(lambda: out.poll(6)[0] == 1)
    time.sleep(0.05)
    assert out.poll(7)[0] == 0
    fseq[0] = 20
    _wait(lambda: out.poll(19)[0] == 1)
    assert m.stop() == 0
    assert m.stats.backpressure > 0 and m.stats.published == 20


def test_mux_overrun_polling():
    """An in producer that laps the mux: the mux resumes from the sequence
    number it found in the line it polled (fd_mux.c:595-603: here line 0
    holds seq 32) and counts the frags it skipped."""
    inl = tile.Link(16, 1232)
    out = tile.Link(64, 1232)
    for i in range(40):                                    # 24 frags overwritten before the mux starts
        inl.publish(b"y" * 10, sig=i)
    m = MuxThread(_mux_cfg([inl], out), tile.MuxCallbacks())
    _wait(lambda: out.poll(7)[0] == 1)
    assert m.stop() == 0
    got = out.drain()
    assert [mt["sig"] for mt, _ in got] == list(range(32, 40))
    assert m.stats.overrun_polling == 32


# ------------------------------------------------- verify tile as callbacks

def _run_vmux(payloads, verifier, seed=0xABCD, batch=4, inflight=2, rr=(0, 1), depth=1 << 12, out_data=None,
              flow=False, consumer=None, cr_max=0, gpu_parse=False):
    inl = tile.Link(depth, 1232)
    outl = tile.Link(depth, tile.TPU_DCACHE_MTU,
                     data_sz=out_data or (len(payloads) + 8) * (tile.TPU_DCACHE_MTU + 64))
    vm = tile.VerifyMuxTile(inl, outl, verifier, hashmap_seed=seed, batch_txn_max=batch, inflight_max=inflight,
                            round_robin_idx=rr[0], round_robin_cnt=rr[1], log_max=1 << 16, flow_control=flow,
                            batch_wait_us=100, cr_max=cr_max, gpu_parse=gpu_parse)
    for p in payloads:
        inl.publish(p)
    th = None
    if consumer is not None:
        th = threading.Thread(target=consumer, args=(outl,), daemon=True)
        th.start()
    vm.run(len(payloads), timeout_s=60)
    if th is not None:
        th.join(30)
    return vm, inl, outl


@pytest.mark.parametrize("gpu_parse", [False, True, 2])
@pytest.mark.parametrize("batch,inflight,lag,rr", [(1, 1, 0, (0, 1)), (7, 2, 2, (0, 1)), (64, 3, 1, (1, 3)),
                                                    (1000, 2, 0, (0, 1))])
def test_vmux_vs_sequential_model(oracle, batch, inflight, lag, rr, gpu_parse):
    """The verify tile as mux callbacks produces the reference loop's outcome
    for every frag and the same published stream (sig = tag, payload,
    fd_txn_t trailer), for any batch size / batches in flight / verifier
    latency / round-robin share -- with fd_txn_parse on the tile's core, and
    with the parse handed to the verifier (gpu_parse: the tile reserves each
    trailer from the payload's counts; here a host stand-in of
    fdgpu_submit_frags parses), and with the payload copy handed over too
    (gpu_parse 2: the tile reserves the out frag from the size alone, the
    verifier -- a host stand-in of fdgpu_submit_frags_io -- reads the
    payload in the in dcache and writes the out frag)."""
    ps = _mixed_stream(800, seed=batch * 17 + lag)
    seed = 0x99 + batch
    ver = tile.PyVerifier(oracle_fn(oracle), slots=inflight, lag=lag)
    vm, _, outl = _run_vmux(ps, ver, seed=seed, batch=batch, inflight=inflight, rr=rr, gpu_parse=gpu_parse)
    exp_out, exp_pub = tile_model.verify_tile_model(ps, seed, oracle_fn(oracle), rr_idx=rr[0], rr_cnt=rr[1])
    seqs, codes = vm.log()
    assert seqs.tolist() == list(range(len(ps)))
    assert codes.tolist() == exp_out
    outs = outl.drain()
    assert [(m["sig"], tile.split_verify_output(f)[0]) for m, f in outs] == [(t, p) for p, _, t in exp_pub]
    assert [tile.split_verify_output(f)[1] for _, f in outs] == [raw for _, raw, _ in exp_pub]
    assert all(m["ctl"] == 0 for m, _ in outs)
    st = vm.stats()
    assert st["published"] == exp_out.count(0) and st["dedup"] == exp_out.count(-2)
    assert st["verify_failed"] == exp_out.count(-1) and st["parse_fail"] == exp_out.count(1)
    assert st["filtered_rr"] == exp_out.count(2)
    assert vm.idle()
    vm.close()


@pytest.mark.parametrize("gpu_parse", [False, True, 2])
def test_vmux_batches_complete_out_of_order(oracle, gpu_parse):
    """Batches finish out of order on the GPU (each ring slot is a stream of
    its own): every 4th batch stays pending for 200 polls while the three
    after it complete at once.  The tile polls the ones behind the oldest
    too (their slots are freed for new batches) but publishes strictly in
    ingest order: outcomes and published stream equal the sequential
    model's, with the out-of-order completions recorded by the verifier."""
    ps = _mixed_stream(900, seed=0x0F0 + int(gpu_parse))
    seed = 0x4242
    ver = tile.PyVerifier(oracle_fn(oracle), slots=4, lag_fn=lambda k: 200 if k % 4 == 0 else 0)
    vm, _, outl = _run_vmux(ps, ver, seed=seed, batch=16, inflight=4, gpu_parse=gpu_parse)
    exp_out, exp_pub = tile_model.verify_tile_model(ps, seed, oracle_fn(oracle))
    seqs, codes = vm.log()
    assert seqs.tolist() == list(range(len(ps)))
    assert codes.tolist() == exp_out
    outs = outl.drain()
    assert [(m["sig"], tile.split_verify_output(f)[0]) for m, f in outs] == [(t, p) for p, _, t in exp_pub]
    assert [tile.split_verify_output(f)[1] for _, f in outs] == [raw for _, raw, _ in exp_pub]
    assert any(b < a for a, b in zip(ver.done, ver.done[1:])), ver.done[:20]   # completed out of order
    # the links were filled before the tile started: it catches up only at
    # the end of the stream, so every batch but the last went out full
    # (its timer alone does not flush a batch while frags are waiting)
    assert ver.batches[:-1] == [16] * (len(ver.batches) - 1) and 0 < ver.batches[-1] <= 16, ver.batches
    assert vm.idle()
    vm.close()


@pytest.mark.parametrize("gpu_parse", [False, True, 2])
def test_vmux_small_dcache_wraps_under_flow_control(oracle, gpu_parse):
    """An out dcache with room for ~8 maximal frags, 12 credits, and a slow
    consumer that reads each published frag (then advances the fseq) while
    the tile runs: the tile wraps the ring many times, stops taking frags
    while the region it would write still holds a frag the consumer may
    read, stops publishing without credits, and every frag the consumer sees
    is intact and in model order."""
    ps = _mixed_stream(600, seed=5)
    seed = 0x5151
    exp_out, exp_pub = tile_model.verify_tile_model(ps, seed, oracle_fn(oracle))
    seen = []

    def consumer(outl):
        seq = outl.seq0
        t0 = time.time()
        while len(seen) < len(exp_pub) and time.time() - t0 < 60:
            rc, meta, _ = outl.poll(seq)
            if rc != 1:
                time.sleep(0.0002)
                continue
            seen.append((meta["sig"], outl.payload(meta)))
            seq += 1
            if random.random() < 0.3:
                time.sleep(0.002)                          # a slow consumer
            outl.fseq[0] = seq

    ver = tile.PyVerifier(oracle_fn(oracle), slots=2, lag=1)
    vm, _, outl = _run_vmux(ps, ver, seed=seed, batch=16, inflight=2, depth=1 << 10,
                            out_data=8 * (tile.TPU_DCACHE_MTU + 64), flow=True, consumer=consumer, cr_max=12,
                            gpu_parse=gpu_parse)
    assert len(seen) == len(exp_pub)
    for (sig, frag), (p, raw, tag) in zip(seen, exp_pub):
        assert sig == tag
        pay, traw = tile.split_verify_output(frag)
        assert pay == p and traw == raw
    seqs, codes = vm.log()
    assert codes.tolist() == exp_out
    assert vm.stats()["backpressure"] > 0 and vm.mux_stats()["backpressure"] > 0
    vm.close()


def test_vmux_gather_drops_lapped_frags(oracle):
    """gpu_parse 2: the verifier reads payloads in the in dcache after the
    tile took them, so the tile re-checks the in mcache once the batch is
    polled; frags whose line the producer lapped meanwhile are dropped as
    overrun (logged LOST), the rest of the stream is verified as the model
    says."""
    ps = _mixed_stream(64, seed=11)[:24]
    assert len(ps) == 24
    inl = tile.Link(16, 1232)
    outl = tile.Link(64, tile.TPU_DCACHE_MTU, data_sz=64 * (tile.TPU_DCACHE_MTU + 64))
    ver = tile.PyVerifier(oracle_fn(oracle), slots=1, lag=1 << 60)       # pending until released below
    vm = tile.VerifyMuxTile(inl, outl, ver, hashmap_seed=0x77, batch_txn_max=8, inflight_max=1, log_max=1 << 10,
                            batch_wait_us=100, gpu_parse=2)
    for p in ps[:8]:
        inl.publish(p)
    vm.start()
    _wait(lambda: len(ver.batches) == 1)                   # the first 8 frags are in flight
    for p in ps[8:]:
        inl.publish(p)                                     # seqs 16..23 overwrite the lines of seqs 0..7
    ver.lag = 0
    _wait(lambda: vm.final_cnt() == len(ps))
    vm.stop()
    seqs, codes = vm.log()
    assert seqs.tolist() == list(range(len(ps)))
    assert codes.tolist()[:8] == [3] * 8                   # FDGPU_VTILE_LOG_LOST
    exp_out, _ = tile_model.verify_tile_model(ps, 0x77, oracle_fn(oracle))
    tail_out, _ = tile_model.verify_tile_model(ps[8:], 0x77, oracle_fn(oracle))
    assert codes.tolist()[8:] == tail_out
    assert vm.stats()["overrun"] == 8 and vm.stats()["lap_margin_min"] == 0     # the first batch was lapped
    vm.close()


def test_vmux_gather_lap_margin(oracle):
    """gpu_parse 2: when a batch is seen complete the tile records how many
    more publishes its oldest frag of each link had left before the producer
    reuses that frag's line (the lap margin a run kept).
    A batch of seqs 0..7 on a 64-deep link completes after the producer has
    published seq 17: seq 0's line is reused by seq 64, so 46 publishes were
    left."""
    ps = _mixed_stream(64, seed=12)[:18]
    inl = tile.Link(64, 1232)
    outl = tile.Link(64, tile.TPU_DCACHE_MTU, data_sz=64 * (tile.TPU_DCACHE_MTU + 64))
    ver = tile.PyVerifier(oracle_fn(oracle), slots=1, lag=1 << 60)       # pending until released below
    vm = tile.VerifyMuxTile(inl, outl, ver, hashmap_seed=0x76, batch_txn_max=8, inflight_max=1, log_max=1 << 10,
                            batch_wait_us=100, gpu_parse=2)
    assert vm.stats()["lap_margin_min"] == 2 ** 64 - 1                     # none measured yet
    for p in ps[:8]:
        inl.publish(p)
    vm.start()
    _wait(lambda: len(ver.batches) == 1)
    for p in ps[8:]:
        inl.publish(p)
    _wait(lambda: vm.stats()["in_frags"] == 16)            # the next batch (8..15) is closed and waits
    ver.lag = 0
    _wait(lambda: vm.final_cnt() == len(ps))
    vm.stop()
    assert vm.stats()["lap_margin_min"] == 46
    vm.close()


def test_vmux_gather_lap_guard_rescues_waiting_frags(oracle):
    """gpu_parse 2, the lap guard: a closed batch that cannot go out (its one
    verifier slot busy) while the producer keeps publishing -- the quic ->
    verify link never waits -- has its frags copied on the tile's core once
    the producer gets within lap_margin (depth / 4) publishes of their lines,
    and the verifier then reads those copies: they are verified as the model
    says.  The in-flight batch's frags whose lines were republished before
    the (late) read are dropped as lapped, and only those."""
    ps = _mixed_stream(200, seed=21)[:70]
    assert len(ps) == 70
    inl = tile.Link(64, 1232)
    outl = tile.Link(256, tile.TPU_DCACHE_MTU, data_sz=256 * (tile.TPU_DCACHE_MTU + 64))
    ver = tile.PyVerifier(oracle_fn(oracle), slots=1, lag=1 << 60)       # pending until released below
    vm = tile.VerifyMuxTile(inl, outl, ver, hashmap_seed=0x78, batch_txn_max=16, inflight_max=1, log_max=1 << 10,
                            batch_wait_us=100, gpu_parse=2)
    for p in ps[:16]:
        inl.publish(p)
    vm.start()
    _wait(lambda: len(ver.batches) == 1)                    # seqs 0..15 in flight, not yet read
    for p in ps[16:32]:
        inl.publish(p)                                      # seqs 16..31: the next batch, closed, waiting
    _wait(lambda: vm.stats()["in_frags"] == 32)
    assert vm.stats()["rescued"] == 0
    for p in ps[32:]:
        inl.publish(p)                                      # up to seq 69: lines 0..5 reused, and the
    _wait(lambda: vm.stats()["rescued"] == 6)               # producer within 16 of lines 16..21's reuse
    time.sleep(0.05)
    assert vm.stats()["rescued"] == 6
    ver.lag = 0
    _wait(lambda: vm.final_cnt() == len(ps))
    vm.stop()
    seqs, codes = vm.log()
    assert seqs.tolist() == list(range(len(ps)))
    assert codes.tolist()[:6] == [3] * 6                    # FDGPU_VTILE_LOG_LOST: lapped before the read
    tail_out, tail_pub = tile_model.verify_tile_model(ps[6:], 0x78, oracle_fn(oracle), seq0=6)
    assert codes.tolist()[6:] == tail_out
    outs = outl.drain()
    assert [(m["sig"], tile.split_verify_output(f)) for m, f in outs] == [(t, (p, raw)) for p, raw, t in tail_pub]
    st = vm.stats()
    assert st["lapped"] == st["overrun"] == 6 and st["rescued"] == 6
    vm.close()


def test_vmux_gather_span_cap_closes_batches(oracle):
    """gpu_parse 2: a batch closes once it spans lap_span_max seqs of a link
    (default depth / 2), whatever its txn cap: 4 round-robin tiles' shares of
    a 64-deep link go out as batches of at most 32 / 4 frags each.  (The
    stand-in reads each batch's payloads at submit, as the device does soon
    after; when the tile polls does not matter here.)"""
    ps = _mixed_stream(400, seed=23)
    inl = tile.Link(64, 1232)
    outl = tile.Link(1 << 10, tile.TPU_DCACHE_MTU, data_sz=(len(ps) + 8) * (tile.TPU_DCACHE_MTU + 64))
    ver = tile.PyVerifier(oracle_fn(oracle), slots=4, read_at_submit=True)
    vm = tile.VerifyMuxTile(inl, outl, ver, hashmap_seed=0x79, batch_txn_max=1000, inflight_max=4, log_max=1 << 12,
                            batch_wait_us=1e6, round_robin_idx=1, round_robin_cnt=4, gpu_parse=2)
    vm.start()
    for k in range(0, len(ps), 40):                         # in steps the tile keeps up with: nothing lapped
        for p in ps[k:k + 40]:
            inl.publish(p)
        _wait(lambda: vm.stats()["in_frags"] == min(k + 40, len(ps)))
    _wait(lambda: vm.final_cnt() == len(ps))
    vm.stop()
    assert ver.batches and max(ver.batches) <= 8 and sum(ver.batches) == len(range(1, len(ps), 4))
    exp_out, _ = tile_model.verify_tile_model(ps, 0x79, oracle_fn(oracle), rr_idx=1, rr_cnt=4)
    assert vm.log()[1].tolist() == exp_out
    vm.close()


def test_vmux_gather_refuses_a_shallow_in_dcache():
    """gpu_parse 2 needs each in dcache to hold depth + 1 maximal frags (so an
    unlapped line means an intact payload): a smaller one is refused."""
    ver = tile.PyVerifier(lambda a, t: np.zeros(len(t), dtype=np.int8))
    outl = tile.Link(64, tile.TPU_DCACHE_MTU, data_sz=tile.vmux_dcache_data_sz(64, 16, 2))
    small = tile.Link(64, 1232, data_sz=40 * 1280)
    with pytest.raises(RuntimeError):
        tile.VerifyMuxTile(small, outl, ver, batch_txn_max=16, gpu_parse=2)
    tile.VerifyMuxTile(small, outl, ver, batch_txn_max=16, gpu_parse=1).close()     # copy modes read at once
    tile.VerifyMuxTile(tile.Link(64, 1232), outl, ver, batch_txn_max=16, gpu_parse=2).close()


def test_frag_out_cap_bounds_every_parse(quic_corpus):
    """fdgpu_frag_out_cap(sz) (the gather tile's reservation, from the size
    alone) holds [payload][pad][fd_txn_t][u16] for every payload that
    parses: the QUIC corpus, generated cfg1/cfg3 txns and random byte
    mutations of them."""
    from firedancer_amd import _lib, workload
    L = _lib.lib()
    rng = random.Random(3)
    pays = list(quic_corpus)
    for gen in (workload.cfg1, workload.cfg3):
        a, t, _ = gen(300, seed=9)
        pays += workload.payloads(a, t)
    muts = []
    for p in pays[:600]:
        for _ in range(6):
            b = bytearray(p)
            b[rng.randrange(len(b))] = rng.randrange(256)
            muts.append(bytes(b))
    checked = 0
    for p in pays + muts:
        fp, _ = tile.txn_parse(p)
        if fp:
            assert ((len(p) + 1) & ~1) + fp + 2 <= L.fdgpu_frag_out_cap(len(p)), (len(p), fp)
            checked += 1
    assert checked > 1000
    assert L.fdgpu_frag_out_cap(1232) <= 1232 + 852 + 2


def test_vmux_cfg_checks():
    inl = tile.Link(64, 1232)
    outl = tile.Link(64, tile.TPU_DCACHE_MTU)
    ver = tile.PyVerifier(lambda a, t: np.zeros(len(t), dtype=np.int8))
    with pytest.raises(RuntimeError):
        tile.VerifyMuxTile(inl, outl, ver, batch_txn_max=0)
    tiny = tile.Link(4, 64)                               # ring smaller than two maximal frags
    with pytest.raises(RuntimeError):
        tile.VerifyMuxTile(inl, tiny, ver, batch_txn_max=4)
    assert tile.vmux_dcache_data_sz(64, 16, 2) >= (64 + 3 * 16) * tile.TPU_DCACHE_MTU


def test_histf_matches_reference_buckets():
    """fdt_histf_init / fdt_histf_sample restate fd_histf (src/util/hist/
    fd_histf.h:77-117,131-158): the header's own example -- min 1, max 100 --
    has exactly these left edges, and a sample lands in [left, right)."""
    h = tile.Histf()
    L = tile.lib()
    L.fdt_histf_init(c.byref(h), 1, 100)
    assert list(h.left_edge)[:16] == [0, 1, 2, 3, 4, 5, 7, 9, 12, 16, 22, 30, 41, 55, 74, 100]
    for v in (0, 1, 6, 99, 100, 10 ** 9):
        L.fdt_histf_sample(c.byref(h), v)
    assert h.counts[0] == 1 and h.counts[1] == 1 and h.counts[5] == 1 and h.counts[14] == 1 and h.counts[15] == 2
    assert h.sum == 0 + 1 + 6 + 99 + 100 + 10 ** 9


def test_vmux_reference_metrics(oracle):
    """The mux loop's metrics in the reference's schema (metrics.xml Link in,
    Stem, Tile; fd_mux.c:597-697): per in link, the consumed frags split into
    published (after_frag kept it) and filtered (after_frag dropped it: here
    the host parse's failures) with their byte counts; before_frag's
    round-robin drops count in no link counter, only in their loop
    histogram; every handled / filtered frag's size is in the size
    histograms; no overrun."""
    ps = _mixed_stream(600, seed=41)
    ver = tile.PyVerifier(oracle_fn(oracle), slots=2)
    inl = tile.Link(1 << 12, 1232)
    outl = tile.Link(1 << 12, tile.TPU_DCACHE_MTU, data_sz=(len(ps) + 8) * (tile.TPU_DCACHE_MTU + 64))
    vm = tile.VerifyMuxTile(inl, outl, ver, hashmap_seed=0x42, batch_txn_max=32, inflight_max=2, log_max=1 << 12,
                            round_robin_idx=1, round_robin_cnt=3, batch_wait_us=100, metrics=True)
    for p in ps:
        inl.publish(p)
    vm.run(len(ps), timeout_s=60)
    m = vm.metrics()
    exp_out, _ = tile_model.verify_tile_model(ps, 0x42, oracle_fn(oracle), rr_idx=1, rr_cnt=3)
    own = [p for k, p in enumerate(ps) if k % 3 == 1]
    failed = [p for k, p in enumerate(ps) if k % 3 == 1 and exp_out[k] == tile.LOG_PARSE_FAIL]
    li = m["link_in"][0]
    assert li["published_count"] + li["filtered_count"] == len(own)
    assert li["filtered_count"] == len(failed) > 0
    assert li["filtered_size_bytes"] == sum(len(p) for p in failed)
    assert li["published_size_bytes"] == sum(len(p) for p in own) - li["filtered_size_bytes"]
    assert li["overrun_polling_count"] == li["overrun_reading_count"] == 0
    assert sum(m["fragment_handled_size_bytes"]["counts"]) == li["published_count"]
    assert sum(m["fragment_filtered_size_bytes"]["counts"]) == li["filtered_count"]
    assert sum(m["loop_filter_before_fragment_duration_ticks"]["counts"]) == len(ps) - len(own)
    assert sum(m["loop_caught_up_duration_ticks"]["counts"]) > 0 and m["housekeeping_cnt"] > 0
    assert m["tick_per_ns"] > 0.1 and m["tile_tid"] > 0 and m["stem_in_backpressure"] == 0
    vm.close()


def test_vmux_metrics_snapshots_are_consistent(oracle):
    """the loop's metrics copy is a seqlock.  Snapshots taken
    while the tile runs are each internally consistent -- the handled-size
    histogram holds exactly the link's published count, the filtered one its
    filtered count -- and the counters never go backwards between them."""
    import threading
    ps = _mixed_stream(4000, seed=43)
    ver = tile.PyVerifier(oracle_fn(oracle), slots=2)
    inl = tile.Link(1 << 13, 1232)
    outl = tile.Link(1 << 13, tile.TPU_DCACHE_MTU, data_sz=(len(ps) + 8) * (tile.TPU_DCACHE_MTU + 64))
    vm = tile.VerifyMuxTile(inl, outl, ver, hashmap_seed=0x43, batch_txn_max=64, inflight_max=2,
                            batch_wait_us=50, metrics=True, lazy_iters=1)
    snaps, stop = [], threading.Event()

    def watch():
        while not stop.is_set():
            snaps.append(vm.metrics())

    th = threading.Thread(target=watch)
    for p in ps:
        inl.publish(p)
    th.start()
    try:
        vm.run(len(ps), timeout_s=60)
    finally:
        stop.set()
        th.join()
    snaps.append(vm.metrics())
    assert len(snaps) > 5
    last = (0, 0, 0)
    for m in snaps:
        li = m["link_in"][0]
        assert sum(m["fragment_handled_size_bytes"]["counts"]) == li["published_count"]
        assert sum(m["fragment_filtered_size_bytes"]["counts"]) == li["filtered_count"]
        cur = (m["housekeeping_cnt"], li["published_count"], li["filtered_count"])
        assert all(a >= b for a, b in zip(cur, last))
        last = cur
    assert last[1] + last[2] == len(ps)
    vm.close()
