"""Engine services on the GPU: the synchronous API's call coalescing, the
completion-word poll's fallback to the runtime event, reference-counted host
registration, slot workspaces that grow with the batches or are reserved up
front.  (The synchronous API's failure policy is tests/test_abi.py's: it
needs no GPU.)  Codes are checked against the golden vectors / the
workload's own labels (bit-exact; no tolerance applies)."""
import ctypes
import os
import threading

import numpy as np
import pytest

from firedancer_amd import _lib, workload
import firedancer_amd as fa

pytestmark = pytest.mark.gpu


def test_sync_api_coalesces_concurrent_callers(vectors):
    """fd_ed25519_verify from 32 threads: every code equals the golden one
    (fd_ed25519_user.c:135-230), and the calls share GPU round trips."""
    vs = vectors["vectors"][:256]
    recs = [(bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["pub"]), v["code"]) for v in vs]
    before = fa.ed25519.sync_stats()
    bad = []

    def worker(k):
        for j in range(k, len(recs), 32):
            m, s, p, code = recs[j]
            got = fa.verify(m, s, p)
            if got != code:
                bad.append((j, got, code))
    ths = [threading.Thread(target=worker, args=(k,)) for k in range(32)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    after = fa.ed25519.sync_stats()
    assert not bad, bad[:5]
    calls = after["calls"] - before["calls"]
    batches = after["batches"] - before["batches"]
    assert calls == len(recs)
    assert batches < calls, (calls, batches)          # coalesced
    assert after["errors"] == before["errors"]


def test_sync_prefixed_names_equal_reference_names(vectors):
    """fdgpu_ed25519_verify{,_batch_single_msg}: the same calls under names
    that do not clash with the reference's CPU fd_ed25519_user.c."""
    L = _lib.lib()
    for v in vectors["vectors"][:24]:
        m, s, p = (bytes.fromhex(v[k]) for k in ("msg", "sig", "pub"))
        assert L.fdgpu_ed25519_verify(m, len(m), s, p) == v["code"]
    pub, sig = workload.sign(bytes(range(32)), b"batch")
    assert L.fdgpu_ed25519_verify_batch_single_msg(b"batch", 5, sig * 3, pub * 3, 3) == 0
    assert L.fdgpu_ed25519_verify_batch_single_msg(b"batch", 5, sig * 3, pub * 3, 0) == -1
    assert L.fdgpu_ed25519_verify_batch_single_msg(b"batch", 5, sig * 17, pub * 17, 17) == -1


def test_poll_completes_without_the_completion_word():
    """A stream that never writes its completion word (FDGPU_DEBUG_DROP_FLAG:
    what a failed stream looks like to the poll) still finishes through the
    runtime event: a non-blocking poll loop ends with the right codes."""
    os.environ["FDGPU_DEBUG_DROP_FLAG"] = "1"
    try:
        eng = fa.VerifyEngine(0, max_txn=1024, ring_depth=2)
    finally:
        del os.environ["FDGPU_DEBUG_DROP_FLAG"]
    try:
        arena, txns, modes = workload.cfg1(300, seed=21)
        tk = eng.submit(arena, txns)
        got = None
        for _ in range(2_000_000):
            got = eng.poll(tk, blocking=False)
            if got is not None:
                break
        assert got is not None, "poll never completed"
        assert ((got == 0) == (modes == 0)).all()
    finally:
        eng.close()


def test_host_register_references():
    """fdgpu_host_register: a range registered twice needs two unregisters;
    a sub-range of a pinned region shares it; a partly overlapping range is
    refused; batches inside a registered range verify from it."""
    L = _lib.lib()
    eng = fa.VerifyEngine(0, max_txn=1024, ring_depth=2)
    eng2 = fa.VerifyEngine(0, max_txn=1024, ring_depth=2)
    try:
        buf = np.zeros(1 << 22, dtype=np.uint8)
        base = buf.ctypes.data
        assert L.fdgpu_host_register(eng._h, base, buf.nbytes) == 0
        assert L.fdgpu_host_register(eng._h, base, buf.nbytes) == 0          # second reference
        assert L.fdgpu_host_register(eng2._h, base + 8192, 4096) == 0        # inside: shared
        arena, txns, modes = workload.cfg1(500, seed=22)
        buf[:arena.size] = arena
        got = eng.verify_txns(buf[:arena.size], txns)
        assert ((got == 0) == (modes == 0)).all()
        assert L.fdgpu_host_unregister(eng._h, base) == 0
        got = eng.verify_txns(buf[:arena.size], txns)                          # still registered once
        assert ((got == 0) == (modes == 0)).all()
        assert L.fdgpu_host_unregister(eng._h, base) == 0
        assert L.fdgpu_host_unregister(eng._h, base) != 0                      # no reference left
        assert L.fdgpu_host_unregister(eng2._h, base + 8192) == 0
        # partial overlap: pin [base, base + 1 MiB), then ask for [base + 512 KiB, base + 2 MiB)
        assert L.fdgpu_host_register(eng._h, base, 1 << 20) == 0
        assert L.fdgpu_host_register(eng._h, base + (1 << 19), 3 << 19) != 0
        assert L.fdgpu_host_unregister(eng._h, base) == 0
    finally:
        eng.close()
        eng2.close()


def test_default_engine_grows_slot_workspace():
    """A default engine (65,536 txns, 12 signatures per txn accepted) opens
    without sizing 12 x 3.2 KB of workspace per txn, and its slots grow to
    the batches they carry: single- then multi-signature batches verify."""
    eng = fa.VerifyEngine(0)
    try:
        a1, t1, m1 = workload.cfg1(2000, seed=23)
        got = eng.verify_txns(a1, t1)
        assert ((got == 0) == (m1 == 0)).all()
        a3, t3, m3 = workload.cfg3(3000, seed=24)
        got3 = eng.verify_txns(a3, t3)
        assert ((got3 == 0) == (m3 == 0)).all()
        assert int(t3["sig_cnt"].sum()) > 3 * 3000
    finally:
        eng.close()


def test_reserve_sizes_every_slot_before_batches():
    """fdgpu_engine_reserve: every ring slot sized for max_sig up front (the
    frag-batch buffers too), refused while a batch is in flight; batches of
    every shape afterwards verify with the workload's labels."""
    eng = fa.VerifyEngine(0, max_txn=2048, ring_depth=3)
    try:
        eng.reserve()
        a, t, modes = workload.cfg3(2000, seed=0x7E5)
        tk = eng.submit(a, t)
        with pytest.raises(RuntimeError):
            eng.reserve()                                  # a slot holds a batch
        codes = eng.poll(tk, blocking=True)
        assert ((codes == 0) == (modes == 0)).all()
        eng.reserve(1000)                                  # smaller than what is there: no change
        a1, t1, m1 = workload.cfg1(2048, seed=0x7E6)
        assert ((eng.verify_txns(a1, t1) == 0) == (m1 == 0)).all()
        with pytest.raises(RuntimeError):
            eng.reserve(2048 * 12 + 1)                     # beyond max_sig
    finally:
        eng.close()


def test_stamps_variant_codes(tmp_path):
    """The phase-stamps diagnostic build (make stamps) verifies bit-exactly
    like the product build: codes against the oracle in a child process that
    loads it through FDGPU_LIB."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = os.path.join(repo, "build", "stamps", "libfd_ed25519_gpu.so")
    if not os.path.exists(so):
        pytest.fail("stamps build missing: make -C firedancer_amd/csrc stamps")
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import firedancer_amd as fa\n"
        "from firedancer_amd import workload, _lib\n"
        "from oracle import oracle as orc\n"
        "assert _lib.LIB_PATH.endswith('build/stamps/libfd_ed25519_gpu.so')\n"
        "assert hasattr(_lib.lib(), 'fdgpu_debug_stamps')\n"
        "a, t, m = workload.cfg1(3000, seed=31)\n"
        "e = fa.VerifyEngine(0, max_txn=4096)\n"
        "got = e.verify_txns(a, t)\n"
        "assert (got == orc.verify_txns(a, t)).all()\n"
        "e.close(); print('ok')\n") % repo
    env = dict(os.environ, FDGPU_LIB=so)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def test_registered_arena_slack_left_unwritten(oracle):
    """A registered arena is DMA'd as it is and the slack past it on the
    device is not zeroed (fdgpu_engine.cpp submit_slot): the SHA block loads
    mask every byte past the message.  The slot's device arena first holds a
    longer batch of 0xA5 bytes, then a registered arena that ends exactly at
    its last message's last byte: every code equals the oracle's."""
    a, t, _ = workload.cfg1(3000, seed=0x51AC)
    end = int(max((t["msg_off"] + t["msg_sz"]).max(), (t["sig_off"] + 64).max(), (t["pub_off"] + 32).max()))
    eng = fa.VerifyEngine(0, max_txn=4096, max_arena=a.nbytes + 8192, ring_depth=1)
    junk = np.full(a.nbytes + 4096, 0xA5, dtype=np.uint8)
    reg = np.full(end + 4096, 0x5A, dtype=np.uint8)
    reg[:end] = a[:end]
    eng.host_register(reg)
    try:
        eng.poll(eng.submit(junk, t), blocking=True)                       # garbage past `end` on the device
        got = eng.poll(eng.submit(reg[:end], t), blocking=True)
        assert (got == oracle.verify_txns(a, t, nthreads=8)).all()
    finally:
        eng.host_unregister(reg)
        eng.close()


def test_big_ring_batches_on_shared_verify_streams(oracle):
    """Ring batches of >= FDGPU_BIG_SIGS (262,144) signatures verify on the
    engine's two big-batch streams in turn (each after its own uploads; its
    read-back waits for it) while small batches keep their slot streams:
    three 300 K batches in flight at once -- staged, from a registered arena,
    and staged again -- with a small batch between them, every code equal
    to the oracle's on a sample and to the workload's labels throughout."""
    a, t, modes = workload.cfg1(300_000, seed=0xB16)
    a_s, t_s, m_s = workload.cfg1(3000, seed=0xB17)
    eng = fa.VerifyEngine(0, max_txn=300_000, max_arena=a.nbytes + 4096, ring_depth=4)
    reg = np.ascontiguousarray(a).copy()
    eng.host_register(reg)
    try:
        ref = oracle.verify_txns(a, t[:20000], nthreads=8)
        tks = [eng.submit(a, t), eng.submit(reg, t), eng.submit(a_s, t_s), eng.submit(a, t)]
        outs = [eng.poll(tk, blocking=True) for tk in tks]
        for k in (0, 1, 3):
            assert (outs[k][:20000] == ref).all(), k
            assert ((outs[k] == 0) == (modes == 0)).all(), k
        assert ((outs[2] == 0) == (m_s == 0)).all()
    finally:
        eng.host_unregister(reg)
        eng.close()
