"""Verify tile over the real GPU engine(s): the reference's test_verify.c
sequences, a mixed stream against the sequential model (oracle verdicts),
the multi-engine dispatcher, and the concurrent producer path."""
import numpy as np
import pytest

import firedancer_amd as fa
from firedancer_amd import tile, workload
import tile_model

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fixtures(txn_fixtures):
    return {t["name"]: bytes.fromhex(t["payload"]) for t in txn_fixtures}


@pytest.fixture(scope="module")
def engines():
    es = [fa.VerifyEngine(0, max_txn=4096, max_sig=4096 * 12, max_arena=4096 * 1232, ring_depth=2)
          for _ in range(2)]
    yield es
    for e in es:
        e.close()


def _tile(engs, inl, outl, **kw):
    ver = tile.EngineVerifier(engs)
    vt = tile.VerifyTile(inl, outl, ver, **kw)
    vt._ver_keep = ver
    return vt


def test_reference_sequences_on_gpu(engines, fixtures):
    v1, v2 = fixtures["test_verify.valid_txn_1sig"], fixtures["test_verify.valid_txn_2sigs"]
    i2, same1 = fixtures["test_verify.invalid_txn_2sigs"], fixtures["test_verify.invalid_txn_same_1sig"]
    same64 = fixtures["test_verify.invalid_txn_1sig_same_64bit"]
    S, F, D = 0, -1, -2
    for seq, exp in (([v2, v2, v2, v1, v1, v1], [S, D, D, S, D, D]), ([i2, i2], [F, F]),
                     ([same1, v1, same1], [F, S, D]), ([v1, same64], [S, F])):
        inl, outl = tile.Link(64, 1232), tile.Link(64, tile.TPU_DCACHE_MTU)
        vt = _tile(engines[:1], inl, outl, batch_txn_max=4, log_max=64)
        for p in seq:
            inl.publish(p)
        vt.run(len(seq), timeout_s=30)
        assert vt.log()[1].tolist() == exp


def test_mixed_stream_two_engines_vs_model(engines, oracle):
    from test_tile import _mixed_stream
    ps = _mixed_stream(3000, seed=99)
    seed = 0xFEED
    inl, outl = tile.Link(1 << 13, 1232), tile.Link(1 << 13, tile.TPU_DCACHE_MTU)
    vt = _tile(engines, inl, outl, hashmap_seed=seed, batch_txn_max=97, inflight_max=4, log_max=1 << 14)
    for p in ps:
        inl.publish(p)
    vt.run(len(ps), timeout_s=60)
    exp, pub = tile_model.verify_tile_model(ps, seed, lambda a, t: oracle.verify_txns(a, t))
    seqs, codes = vt.log()
    assert codes.tolist() == exp
    outs = outl.drain()
    assert [(m["sig"], tile.split_verify_output(f)[0]) for m, f in outs] == [(t, p) for p, _, t in pub]
    assert vt.stats()["batches"] >= len(ps) // 97


def test_quic_corpus_through_tile(engines, quic_corpus, oracle):
    arena, txns, codes = quic_corpus
    ps = [bytes(arena[int(t["sig_off"]) - 1: int(t["msg_off"]) + int(t["msg_sz"])]) for t in txns]
    inl, outl = tile.Link(1 << 11, 1232), tile.Link(1 << 11, tile.TPU_DCACHE_MTU)
    vt = _tile(engines, inl, outl, batch_txn_max=256, inflight_max=2)
    for p in ps:
        inl.publish(p)
    vt.run(len(ps), timeout_s=60)
    st = vt.stats()
    exp, pub = tile_model.verify_tile_model(ps, 0x5EEDF00D, lambda a, t: oracle.verify_txns(a, t))
    assert st["published"] == len(pub) == exp.count(0) and st["verify_failed"] == 0


def test_producer_at_rate_no_overrun(engines):
    """Producer thread at 500K frags/s into a 2^16-deep link, tile keeping up."""
    a, t, modes = workload.cfg3(20000, seed=7)
    ps = workload.payloads(a, t)
    arena, offs, sizes = workload.pack_payloads(ps)
    inl, outl = tile.Link(1 << 16, 1232), tile.Link(1 << 16, tile.TPU_DCACHE_MTU)
    vt = _tile(engines, inl, outl, batch_txn_max=2048, inflight_max=4, batch_wait_us=100)
    prod = tile.Producer(inl, arena, offs, sizes, rate_tps=500000)
    vt.run(len(ps), timeout_s=60)
    prod.join()
    st = vt.stats()
    assert st["overrun"] == 0 and st["in_frags"] == len(ps)
    assert st["published"] == int((modes == 0).sum())
    lat = vt.latencies_ns()
    assert len(lat) == st["batches"] and np.percentile(lat, 99) < 50e6


def test_twelve_signature_txns_default_config():
    """Engines opened with the default max_sig (12 per txn) and a tile with
    the default signature cap: a stream of 12-signature transactions never
    builds a batch the engine rejects, and matches the sequential model."""
    a3, t3, _ = workload.make_txns(3000, 0x12, multi=True, max_sigs=12, key_pool=4096)
    keep = t3["sig_cnt"] >= 10
    ps = [p for p, k in zip(workload.payloads(a3, t3), keep) if k]
    eng = fa.VerifyEngine(0, max_txn=256, ring_depth=2)
    try:
        inl, outl = tile.Link(1 << 12, 1232), tile.Link(1 << 12, tile.TPU_DCACHE_MTU)
        vt = _tile([eng], inl, outl, batch_txn_max=256, log_max=1 << 13)
        for p in ps:
            inl.publish(p)
        vt.run(len(ps), timeout_s=60)
        from oracle import oracle as orc

        def ofn(arena, txns):
            return orc.verify_txns(arena, txns, nthreads=8)
        exp_out, _ = tile_model.verify_tile_model(ps, 0x5EEDF00D, ofn)
        st = vt.stats()
        assert vt.log()[1].tolist() == exp_out
        assert st["verify_errors"] == 0 and st["sigs"] >= 10 * len(ps)
        vt.close()
    finally:
        eng.close()


# ------------------------------------ the verify tile as mux callbacks (vmux)

@pytest.mark.parametrize("gpu_parse", [False, True, 2])
def test_vmux_mixed_stream_vs_model_gpu(engines, oracle, gpu_parse):
    """fdgpu_vmux on fdt_mux_run over the MI355X engines: frags copied into
    the out dcache (registered with both engines, so each batch is DMA'd from
    there with no staging copy), verified, and published in place -- every
    outcome and the published stream equal the sequential model's.  With
    gpu_parse the batches are frag batches (fdgpu_submit_frags): fd_txn_parse
    runs on the GPU and the trailers come back from it.  With gpu_parse 2
    (fdgpu_submit_frags_io) the GPU reads each payload in the registered in
    dcache and writes the whole out frag back: the tile copies nothing."""
    from test_tile import _mixed_stream
    ps = _mixed_stream(3000, seed=7)
    seed = 0xC0DE
    inl = tile.Link(1 << 13, 1232)
    outl = tile.Link(1 << 13, tile.TPU_DCACHE_MTU, data_sz=tile.vmux_dcache_data_sz(1 << 13, 101, 3))
    ver = tile.EngineVerifier(engines)
    vm = tile.VerifyMuxTile(inl, outl, ver, hashmap_seed=seed, batch_txn_max=101, inflight_max=3, log_max=1 << 14,
                            gpu_parse=gpu_parse)
    for p in ps:
        inl.publish(p)
    vm.run(len(ps), timeout_s=60)
    exp, pub = tile_model.verify_tile_model(ps, seed, lambda a, t: oracle.verify_txns(a, t))
    seqs, codes = vm.log()
    assert seqs.tolist() == list(range(len(ps))) and codes.tolist() == exp
    outs = outl.drain()
    assert [(m["sig"], tile.split_verify_output(f)) for m, f in outs] == [(t, (p, raw)) for p, raw, t in pub]
    st = vm.stats()
    assert st["batches"] >= (len(ps) - st["parse_fail"]) // 101 and vm.idle()
    assert st["verify_errors"] == 0
    vm.close()
    ver.close()


def test_vmux_bench_engine_flags_gpu(oracle):
    """The tile over engines opened as bench.py's tile lines open them
    (FDGPU_FLAG_PAIR_AUTO | FDGPU_FLAG_SPREAD_AUTO): small batches take the
    two-lane kernel, one block per CU; every outcome and the published
    stream (gathered mode: out frags written by the GPU) equal the
    sequential model's."""
    from test_tile import _mixed_stream
    es = [fa.VerifyEngine(0, max_txn=4096, max_sig=4096 * 12, max_arena=4096 * 1232, ring_depth=4, pair_auto=True,
                          spread_auto=True) for _ in range(2)]
    try:
        ps = _mixed_stream(3000, seed=0x51)
        seed = 0xBEEF
        inl = tile.Link(1 << 13, 1232)
        outl = tile.Link(1 << 13, tile.TPU_DCACHE_MTU, data_sz=tile.vmux_dcache_data_sz(1 << 13, 257, 4))
        ver = tile.EngineVerifier(es)
        vm = tile.VerifyMuxTile(inl, outl, ver, hashmap_seed=seed, batch_txn_max=257, inflight_max=4,
                                log_max=1 << 14, gpu_parse=2)
        for p in ps:
            inl.publish(p)
        vm.run(len(ps), timeout_s=60)
        exp, pub = tile_model.verify_tile_model(ps, seed, lambda a, t: oracle.verify_txns(a, t))
        seqs, codes = vm.log()
        assert seqs.tolist() == list(range(len(ps))) and codes.tolist() == exp
        outs = outl.drain()
        assert [(m["sig"], tile.split_verify_output(f)) for m, f in outs] == [(t, (p, raw)) for p, raw, t in pub]
        assert vm.stats()["verify_errors"] == 0 and vm.idle()
        vm.close()
        ver.close()
    finally:
        for e in es:
            e.close()


@pytest.mark.parametrize("gpu_parse", [0, 2])
def test_vmux_two_tiles_share_engines_gpu(engines, oracle, gpu_parse):
    """Two verify mux tiles on their own threads take the round-robin shares
    of one in link (fd_verify.c:46) and share the node's engines (the ring
    API is thread-safe per engine); each tile's outcomes and published
    stream equal the model of its share, with the out dcache wrapping
    several times under flow control from a consumer thread."""
    import threading
    import time
    from test_tile import _mixed_stream
    ps = _mixed_stream(4000, seed=11)
    seed = 0xBEEF
    inl = tile.Link(1 << 13, 1232)
    tiles, outs, vers = [], [], []
    for k in range(2):
        outl = tile.Link(1 << 12, tile.TPU_DCACHE_MTU, data_sz=tile.vmux_dcache_data_sz(64, 64, 2))
        ver = tile.EngineVerifier(engines)
        vm = tile.VerifyMuxTile(inl, outl, ver, hashmap_seed=seed, batch_txn_max=64, inflight_max=2,
                                round_robin_idx=k, round_robin_cnt=2, log_max=1 << 14, cr_max=64,
                                flow_control=True, gpu_parse=gpu_parse)
        tiles.append(vm); outs.append(outl); vers.append(ver)
    seen = [[], []]
    stop = threading.Event()

    def consume(k):
        outl, seq = outs[k], outs[k].seq0
        while not stop.is_set():
            rc, meta, _ = outl.poll(seq)
            if rc != 1:
                time.sleep(0.0001)
                continue
            seen[k].append((meta["sig"], outl.payload(meta)))
            seq += 1
            outl.fseq[0] = seq

    cons = [threading.Thread(target=consume, args=(k,), daemon=True) for k in range(2)]
    for t in cons:
        t.start()
    for p in ps:
        inl.publish(p)
    for vm in tiles:
        vm.start()
    t0 = time.time()
    while any(vm.final_cnt() < len(ps) for vm in tiles):
        assert time.time() - t0 < 60
        time.sleep(0.001)
    for vm in tiles:
        vm.stop()
    time.sleep(0.05)
    stop.set()
    for t in cons:
        t.join(10)
    for k, vm in enumerate(tiles):
        exp, pub = tile_model.verify_tile_model(ps, seed, lambda a, t: oracle.verify_txns(a, t), rr_idx=k,
                                                rr_cnt=2)
        assert vm.log()[1].tolist() == exp
        assert [(s, tile.split_verify_output(f)) for s, f in seen[k]] == [(t, (p, raw)) for p, raw, t in pub]
        vm.close()
        vers[k].close()


# --------------------- the gather tile against a producer that laps it

def _gather_lap_run(engines, oracle, ps, depth, rate, batch, inflight, wait_us, guard):
    """A Producer thread publishes ps at `rate` into a `depth`-deep quic ->
    verify link while the gather-mode mux tile (gpu_parse 2) runs over the
    MI355X: returns the tile's stats and, for the frags it did not lose, its
    outcomes and published stream next to the sequential model's over
    exactly those frags (the lost ones -- lapped before the device read
    them, or skipped by the mux as overrun -- never reach the tcache)."""
    import time
    seed = 0x1AB
    arena, offs, sizes = workload.pack_payloads(ps)
    inl = tile.Link(depth, 1232)
    od = 1 << (len(ps) - 1).bit_length()
    outl = tile.Link(od, tile.TPU_DCACHE_MTU, data_sz=(len(ps) + 64) * (tile.TPU_DCACHE_MTU + 64))
    ver = tile.EngineVerifier(engines[:1])
    kw = {} if guard else dict(lap_span_max=tile.LAP_OFF, lap_margin=tile.LAP_OFF)
    vm = tile.VerifyMuxTile(inl, outl, ver, hashmap_seed=seed, batch_txn_max=batch, inflight_max=inflight,
                            batch_wait_us=wait_us, log_max=1 << 17, gpu_parse=2, **kw)
    try:
        vm.start()
        prod = tile.Producer(inl, arena, offs, sizes, rate_tps=rate)
        n_pub, _ = prod.join()
        assert n_pub == len(ps)
        t0, last = time.time(), -1
        while True:                                   # the tile is done once nothing changes and nothing is held
            time.sleep(0.2)
            cur = vm.final_cnt()
            if cur == last and vm.idle():
                break
            last = cur
            assert time.time() - t0 < 60
        vm.stop()
        st, mst = vm.stats(), vm.mux_stats()
        assert st["corrupt"] == 0 and st["verify_errors"] == 0
        assert vm.final_cnt() + mst["overrun_polling"] + mst["overrun_reading"] == len(ps)
        seqs, codes = vm.log()
        lost = codes == tile.LOG_LOST
        assert int(lost.sum()) == st["lapped"] == st["overrun"]
        kept = seqs[~lost].tolist()
        exp_out, exp_pub = tile_model.verify_tile_model([ps[s] for s in kept], seed,
                                                        lambda a, t: oracle.verify_txns(a, t), seqs=kept)
        assert codes[~lost].tolist() == exp_out
        outs = outl.drain()
        # no torn frag published: every published frag is the model's, payload and trailer
        assert [(m["sig"], tile.split_verify_output(f)) for m, f in outs] == [(t, (p, raw)) for p, raw, t in exp_pub]
        return st, mst, len(kept)
    finally:
        vm.close()
        ver.close()


def test_vmux_gather_drops_frags_lapped_on_device_gpu(engines, oracle):
    """Lap guard off, batches held 3 ms on a 1024-deep link fed at 1 M
    frags/s: the producer laps the oldest frags of every batch before the
    device reads them; the device's re-check of each frag's mcache line
    (fdgpu_submit_frags_io links) drops exactly those as lapped, and every
    other frag is verified, deduplicated and published as the reference loop
    would, with no torn payload published."""
    from test_tile import _mixed_stream
    ps = _mixed_stream(20000, seed=31)
    st, mst, kept = _gather_lap_run(engines, oracle, ps, 1024, 1.0e6, 4096, 3, 3000, guard=False)
    assert st["lapped"] > 1000 and kept > 2000 and st["rescued"] == 0


def test_vmux_gather_lap_guard_gpu(engines, oracle):
    """The same stream with the lap guard on (batches close at depth / 2
    seqs, frags within depth / 4 of being lapped copied by the tile): the
    tile's outcomes and published stream equal the model's over every frag
    it kept, and it keeps nearly all of them.  The link is 2048 deep here:
    at 1 M frags/s a 1024-deep one gives the tile's own thread 1 ms of
    slack, and a shared box's scheduler took that away now and then (the
    mux then skips a whole ring as overrun: 1024 frags it never reads,
    which no guard can protect); batches are still held 3 ms, past the
    link's 2 ms wrap, so the guard has frags to copy."""
    from test_tile import _mixed_stream
    ps = _mixed_stream(20000, seed=31)
    st, mst, kept = _gather_lap_run(engines, oracle, ps, 2048, 1.0e6, 4096, 3, 3000, guard=True)
    assert kept >= len(ps) * 0.95, (st, mst)


def test_vmux_gather_unregistered_mcache_is_fatal_gpu(engines):
    """a gather tile whose in-link mcache was never registered
    with the engines (only the dcaches were) must stop with the engine's
    FDGPU_ERR_UNREG (-14) at its first submit -- not reject every batch as
    malformed while it looks healthy."""
    from test_tile import _mixed_stream
    ps = _mixed_stream(300, seed=5)
    inl = tile.Link(1 << 10, 1232)
    outl = tile.Link(1 << 10, tile.TPU_DCACHE_MTU, data_sz=tile.vmux_dcache_data_sz(1 << 10, 64, 2))
    ver = tile.EngineVerifier(engines[:1])
    vm = tile.VerifyMuxTile(inl, outl, ver, batch_txn_max=64, inflight_max=2, gpu_parse=2, register=False)
    for b in (outl.dcache, inl.dcache):
        engines[0].host_register(b)
    try:
        for p in ps:
            inl.publish(p)
        with pytest.raises(RuntimeError, match="-14"):
            vm.run(len(ps), timeout_s=30)
        st = vm.stats()
        assert st["published"] == 0 and st["verify_errors"] == 0
    finally:
        vm.close()
        ver.close()
        for b in (outl.dcache, inl.dcache):
            engines[0].host_unregister(b)


def test_vmux_gather_reads_reasm_link_gpu(oracle, engines):
    """The gather-mode mux tile on the reference's actual quic -> verify link
    type, the TPU reassembly slot arena (fd_tpu.h:20-45, fd_frankendancer.c:
    59 is_reasm): fragmented streams reassembled and published while the tile
    runs on its thread; the device reads each payload in its slot and
    re-checks the slot's mcache line; outcomes and the published stream equal
    the model's.  A shallow arena with the lap guard off and batches held
    20 ms is lapped (a reused slot is rewritten under the pending batch):
    exactly the lapped frags are dropped, none is published torn."""
    import random
    import time
    from test_tile import _mixed_stream
    for depth, burst, n, guard, wait_us in ((1 << 12, 32, 4000, True, 100), (64, 4, 3000, False, 20000)):
        ps = [p for p in _mixed_stream(n, seed=depth + burst) if len(p) <= 1232]
        rnd = random.Random(depth)
        r = tile.TpuReasm(depth, burst)
        outl = tile.Link(1 << 13, tile.TPU_DCACHE_MTU, data_sz=(len(ps) + 64) * (tile.TPU_DCACHE_MTU + 64))
        ver = tile.EngineVerifier(engines[:1])
        kw = {} if guard else dict(lap_span_max=tile.LAP_OFF, lap_margin=tile.LAP_OFF)
        vm = tile.VerifyMuxTile(r, outl, ver, batch_txn_max=256, inflight_max=2, batch_wait_us=wait_us,
                                log_max=1 << 14, gpu_parse=2, **kw)
        try:
            vm.start()
            i, open_, pub_order = 0, [], []
            while i < len(ps) or open_:
                if i < len(ps) and len(open_) < burst and (not open_ or rnd.random() < 0.5):
                    open_.append([r.prepare(), ps[i], 0])
                    i += 1
                    continue
                k = rnd.randrange(len(open_))
                slot, p, sent = open_[k]
                m = rnd.randrange(1, 400)
                back = rnd.randrange(0, min(sent, 20) + 1)
                assert r.append(slot, p[sent - back:sent + m], sent - back) == tile.REASM_SUCCESS
                open_[k][2] = min(len(p), sent + m)
                if open_[k][2] == len(p):
                    assert r.publish(slot) == tile.REASM_SUCCESS
                    pub_order.append(p)
                    open_.pop(k)
            t0 = time.time()
            last = -1
            while not (vm.idle() and vm.final_cnt() == last):     # (unguarded: the mux may skip lapped seqs)
                last = vm.final_cnt()
                assert time.time() - t0 < 60
                time.sleep(0.1)
            assert vm.final_cnt() == r.next_seq or not guard
            vm.stop()
            st = vm.stats()
            seqs, codes = vm.log()
            if guard:
                assert seqs.tolist() == list(range(r.next_seq))
            lost = codes == tile.LOG_LOST
            assert int(lost.sum()) == st["lapped"]
            kept = seqs[~lost].tolist()
            exp_out, exp_pub = tile_model.verify_tile_model([pub_order[s] for s in kept], 0x5EEDF00D,
                                                            lambda a, t: oracle.verify_txns(a, t), seqs=kept)
            assert codes[~lost].tolist() == exp_out
            outs = outl.drain()
            assert [tile.split_verify_output(f)[0] for _, f in outs] == [p for p, _, _ in exp_pub]
            if guard:
                assert st["lapped"] == 0 and exp_out.count(0) > 100
            else:
                assert st["lapped"] > 0 and len(kept) > 20     # (how many survive is timing: DMA vs load gather)
        finally:
            vm.close()
            ver.close()
