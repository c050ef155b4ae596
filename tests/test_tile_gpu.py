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
