"""Process separation of the verify stage: tango
links in shared memory joined by independent processes, the engine process
(firedancer_amd/engine_proc.py) running the batched verify tile, and the
dedup tile inside the reference's seccomp policy (verify.seccomppolicy /
dedup.seccomppolicy: write + fsync only).  Outputs are checked frag by frag
against the sequential models of the reference loops (tests/tile_model.py).
The CPU tests use the oracle as the engine process's verifier; the GPU test
runs the same pipeline over the MI355X engine."""
import multiprocessing as mp
import os
import signal
import uuid

import pytest

from firedancer_amd import tile
import tile_model
from test_tile import _mixed_stream


def _shm_path(tag):
    return f"/dev/shm/fdgpu_test_{os.getpid()}_{tag}_{uuid.uuid4().hex[:8]}"


def _fork_and_wait(fn):
    pid = os.fork()
    if pid == 0:
        try:
            fn()
        finally:
            os._exit(5)
    _, status = os.waitpid(pid, 0)
    return status


def test_sandbox_allows_log_writes():
    """write(2) and exit pass the policy."""
    def child():
        tile.sandbox_enter(2)
        os.write(2, b"")
        os._exit(0)
    status = _fork_and_wait(child)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0, status


def test_sandbox_kills_other_syscalls():
    """Any other syscall (here openat) kills the process, as the reference's
    generated filters do."""
    def child():
        tile.sandbox_enter(2)
        os.open("/dev/null", os.O_RDONLY)
        os._exit(0)
    status = _fork_and_wait(child)
    assert os.WIFSIGNALED(status) and os.WTERMSIG(status) == signal.SIGSYS, status


def test_shm_link_join_roundtrip():
    """A link formatted in a /dev/shm file is the same link when joined by
    path: publish on one mapping, poll on the other; the consumer fseq is
    shared too."""
    path = _shm_path("rt")
    try:
        a = tile.Link.shm_create(path, 64, 1232, seq0=7)
        b = tile.Link.shm_join(path)
        assert (b.depth, b.mtu, b.seq0, b.wmark) == (64, 1232, 7, a.wmark)
        for i in range(100):                                   # wraps the 64-deep ring
            a.publish(bytes([i % 251]) * (1 + i * 11 % 1200), sig=i)
        got = b.drain(seq=7 + 36)
        assert [m["sig"] for m, _ in got] == list(range(36, 100))
        assert all(p == bytes([m["sig"] % 251]) * (1 + m["sig"] * 11 % 1200) for m, p in got)
        assert b.poll(7)[0] == -1                              # overrun seen by the joiner
        b.fseq[0] = 99
        assert int(a.fseq[0]) == 99
    finally:
        os.unlink(path)


def _pipeline(ps, use_gpu, oracle, batch=64):
    """quic (this process) -> verify (engine process) -> dedup (sandboxed
    child) over three shared-memory links."""
    seed, dseed = 0x5EEDF00D, 0xD5
    paths = [_shm_path(n) for n in ("qv", "vd", "dd")]
    try:
        inl = tile.Link.shm_create(paths[0], 1 << 12, 1232)
        vd = tile.Link.shm_create(paths[1], 1 << 12, tile.TPU_DCACHE_MTU)
        dd = tile.Link.shm_create(paths[2], 1 << 12, tile.TPU_DCACHE_MTU)
        exp_out, exp_pub = tile_model.verify_tile_model(ps, seed, lambda a, t: oracle.verify_txns(a, t))
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        import _engine_proc_worker
        eng = ctx.Process(target=_engine_proc_worker.run,
                          args=(paths[0], paths[1], len(ps), use_gpu, q,
                                dict(hashmap_seed=seed, batch_txn_max=batch, inflight_max=3)))
        eng.start()
        dt = tile.DedupTile([vd], dd, hashmap_seed=dseed, tcache_depth=1 << 14)
        # the sandboxed dedup child is forked only from a process that has not
        # initialised the GPU (GPU test: the dedup tile runs here afterwards)
        pid, dstats = dt.fork_sandboxed(len(exp_pub), idle_s=60.0) if not use_gpu else (None, None)
        for p in ps:
            inl.publish(p)
        kind, st = q.get(timeout=180)
        eng.join(timeout=60)
        assert kind == "ok", st
        if pid is not None:
            _, status = os.waitpid(pid, 0)
            assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0, status
        else:
            dt.run_until_idle()
            dstats = dt.stats
        # verify tile: the reference loop's outcome for every frag
        assert st["published"] == exp_out.count(0) and st["dedup"] == exp_out.count(-2)
        assert st["verify_failed"] == exp_out.count(-1) and st["parse_fail"] == exp_out.count(1)
        vouts = vd.drain()
        assert [(m["sig"], tile.split_verify_output(f)[0]) for m, f in vouts] == [(t, p) for p, _, t in exp_pub]
        # sandboxed dedup tile: every verified txn once, sig 0
        exp_d = tile_model.dedup_model([f for _, f in vouts], dseed, 1 << 14)
        got = dd.drain()
        assert [f for _, f in got] == exp_d and all(m["sig"] == 0 for m, _ in got)
        ds = dstats()
        assert ds["in_frags"] == len(vouts) and ds["published"] == len(exp_d) and ds["overrun"] == 0
        return exp_out
    finally:
        for p in paths:
            if os.path.exists(p):
                os.unlink(p)


def test_engine_process_pipeline_cpu(oracle):
    ps = _mixed_stream(600, seed=71)
    exp_out = _pipeline(ps, False, oracle)
    assert exp_out.count(-2) > 10 and exp_out.count(-1) > 10


@pytest.mark.gpu
def test_engine_process_pipeline_gpu(oracle):
    ps = _mixed_stream(3000, seed=72)
    exp_out = _pipeline(ps, True, oracle, batch=512)
    assert exp_out.count(0) > 1000


@pytest.mark.gpu
def test_engine_process_cli_gpu(oracle):
    """`python -m firedancer_amd.engine_proc` as an operator starts it: joins
    the links by path, verifies on the GPU, prints the tile's stats."""
    import json
    import subprocess
    import sys
    ps = _mixed_stream(1500, seed=73)
    paths = [_shm_path(n) for n in ("qv", "vd")]
    try:
        inl = tile.Link.shm_create(paths[0], 1 << 12, 1232)
        vd = tile.Link.shm_create(paths[1], 1 << 12, tile.TPU_DCACHE_MTU)
        for p in ps:
            inl.publish(p)
        r = subprocess.run([sys.executable, "-m", "firedancer_amd.engine_proc", "--in", paths[0], "--out", paths[1],
                            "--frags", str(len(ps)), "--batch", "512", "--timeout", "60"],
                           capture_output=True, text=True, timeout=120,
                           cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        assert r.returncode == 0, r.stderr[-2000:]
        st = json.loads(r.stdout.strip().splitlines()[-1])
        exp_out, exp_pub = tile_model.verify_tile_model(ps, 0x5EEDF00D, lambda a, t: oracle.verify_txns(a, t))
        assert st["published"] == exp_out.count(0) and st["verify_failed"] == exp_out.count(-1)
        assert [m["sig"] for m, _ in vd.drain()] == [t for _, _, t in exp_pub]
    finally:
        for p in paths:
            if os.path.exists(p):
                os.unlink(p)
