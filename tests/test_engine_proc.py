"""Process separation of the verify stage, in the
shape the reference's topology runs it (fd_frankendancer.c:59-60,131-133,
fd_topo_run.c:50-171): tango links in shared memory (every page faulted in
before use), a producer process publishing into the quic -> verify link
(tools/quic_feed.py), the engine process (firedancer_amd/engine_proc.py)
running the gather-mode verify mux tile -- the tile every bench number comes
from -- over that link, and the dedup tile in a process of its own inside
the reference's seccomp policy (verify.seccomppolicy / dedup.seccomppolicy:
write + fsync only).  tools/xproc.py launches the three.  Outputs are
checked frag by frag against the sequential models of the reference loops
(tests/tile_model.py).  The CPU tests run the engine process's loop over the
oracle (tests/_engine_proc_worker.py); the GPU tests over the MI355X."""
import os
import signal
import sys
import uuid

import pytest

import numpy as np

from firedancer_amd import tile, workload
import tile_model
from test_tile import _mixed_stream

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import xproc  # noqa: E402

CPU_ENGINE = [sys.executable, os.path.join(REPO, "tests", "_engine_proc_worker.py")]


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
    """write(2) and exit pass the policy.  After entry the child only makes
    the raw calls through functions bound beforehand, with the collector off:
    under the tiles' policy even an mmap of a new allocator arena kills the
    process (the sanitizer build's allocator takes one at times), and a
    Python-level write could be the call that needs it."""
    def child():
        import ctypes
        import gc
        libc = ctypes.CDLL(None)
        sc = libc.syscall
        sc.restype, sc.argtypes = ctypes.c_long, [ctypes.c_long] * 4
        enter = tile.lib().fdt_sandbox_enter
        nr_write, nr_exit_group = 1, 231
        gc.disable()
        rc = enter(2)
        wr = sc(nr_write, 2, 0, 0)                      # a 0-byte write to fd 2
        sc(nr_exit_group, 0 if rc == 0 and wr == 0 else 7, 0, 0)
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


def test_engine_sandbox_kills_open():
    """The engine process's policy (fdt_sandbox_engine_enter, every thread):
    the calls a running engine makes pass -- memory, futexes, clocks, a
    thread, writes -- and opening a file kills the process with SIGSYS."""
    def child():
        import threading
        tile.engine_sandbox_enter()
        buf = np.zeros(1 << 22, dtype=np.uint8)            # mmap / munmap
        th = threading.Thread(target=lambda: buf.sum())   # clone (a thread), futex
        th.start()
        th.join()
        os.write(2, b"")
        os.open("/dev/null", os.O_RDONLY)
        os._exit(0)
    status = _fork_and_wait(child)
    assert os.WIFSIGNALED(status) and os.WTERMSIG(status) == signal.SIGSYS, status


def test_engine_sandbox_report_mode():
    """Report mode refuses the same calls without killing: open fails with
    EPERM and is listed; a process (fork) is refused too; ioctl is refused on
    an fd that is not the GPU driver's; a signal to another process (tgkill
    of the parent) is refused while one to the process's own thread passes."""
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:
        try:
            import ctypes
            import fcntl
            import resource
            import termios
            import threading
            libc = ctypes.CDLL(None, use_errno=True)

            def prctl_dumpable():                               # PR_SET_DUMPABLE (4): refused
                if libc.prctl(4, 1, 0, 0, 0) != 0:
                    raise OSError(ctypes.get_errno(), "prctl")
            def tgkill_parent():                                # a signal (0) to another process: refused
                if libc.syscall(234, os.getppid(), os.getppid(), 0) != 0:
                    raise OSError(ctypes.get_errno(), "tgkill")
            tile.engine_sandbox_enter(report=True)
            os.fstat(w)                                         # fstat of a held fd: allowed
            signal.pthread_kill(threading.get_ident(), 0)      # tgkill within the process: allowed
            libc.prctl(15, b"engine-test", 0, 0, 0)             # PR_SET_NAME: allowed
            errs = []
            resource.getrlimit(resource.RLIMIT_NOFILE)            # prlimit64 of itself, reading: allowed
            for what in (lambda: os.open("/dev/null", os.O_RDONLY), os.fork,
                         lambda: fcntl.ioctl(0, termios.FIONREAD, b"    "),
                         lambda: resource.setrlimit(resource.RLIMIT_NOFILE, resource.getrlimit(resource.RLIMIT_NOFILE)),
                         lambda: resource.prlimit(os.getppid(), resource.RLIMIT_NOFILE),
                         lambda: os.stat("/etc"), prctl_dumpable, tgkill_parent):
                try:
                    what()
                    errs.append("allowed")
                except (OSError, ValueError) as e:          # (setrlimit reports EPERM as ValueError)
                    errs.append(getattr(e, "errno", None) or 1)
            n, names = tile.engine_sandbox_report()
            os.write(w, repr((errs, n, names)).encode())
        finally:
            os._exit(0)
    os.close(w)
    _, status = os.waitpid(pid, 0)
    errs, n, names = eval(os.read(r, 4096).decode())
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0, status
    assert errs == [1] * 8 and n == 8, (errs, n)
    assert "openat" in names and "ioctl" in names and ("clone" in names or "fork" in names), names
    assert "prlimit64" in names and "newfstatat" in names and "prctl" in names, names
    assert "tgkill" in names, names


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


def _npz(tmp_path, ps):
    arena, offs, sizes = workload.pack_payloads(ps)
    p = str(tmp_path / "frags.npz")
    np.savez(p, arena=arena, offs=offs, sizes=sizes)
    return p


def _sig0(f):
    payload, raw = tile.split_verify_output(f)
    so = tile.txn_decode(raw)["signature_off"]
    return payload[so:so + 64]


def _check_dedup_multi_link(tile_outs, dedup_out):
    """The dedup tile over several verify -> dedup links: which link it
    services first is a matter of timing (the mux's round robin over ready
    links), so the check is by content: with the reference's tcache depth
    (4,194,302, far above these streams) every distinct first signature the
    verify tiles published comes out exactly once, as one of the frags that
    carried it, and the frags of each link keep that link's order."""
    by_sig = {}
    for k, frags in enumerate(tile_outs):
        for j, f in enumerate(frags):
            by_sig.setdefault(_sig0(f), []).append((k, j, f))
    got = [_sig0(f) for f in dedup_out]
    assert len(got) == len(set(got)) == len(by_sig)
    pos = {k: -1 for k in range(len(tile_outs))}
    for f, s in zip(dedup_out, got):
        src = [(k, j) for k, j, g in by_sig[s] if g == f]
        assert src, "dedup published a frag no verify tile published"
        if len(by_sig[s]) == 1:                       # carried by one link only: that link's order holds
            k, j = src[0]
            assert j > pos[k]
            pos[k] = j


def _xproc_vs_model(tmp_path, ps, oracle, tiles=1, dedup=True, engine_cmd=None, engine_procs=1, **kw):
    """producer process -> engine process(es) (T gather-mode mux tiles, round
    robin over one quic -> verify link; with engine_procs=E, E processes of
    T/E tiles each take global shares rr_idx..rr_idx+T/E-1 of T) ->
    sandboxed dedup process; every frag's outcome, every tile's published
    stream and the dedup tile's output against the sequential models."""
    seed, dseed = 0x5EEDF00D, 0xD5
    exp = [tile_model.verify_tile_model(ps, seed, lambda a, t: oracle.verify_txns(a, t), rr_idx=k, rr_cnt=tiles)
           for k in range(tiles)]
    n_pub = sum(len(pub) for _, pub in exp)
    res = xproc.run(_npz(tmp_path, ps), len(ps), tiles=tiles, producers=1, seed=seed, dedup=dedup,
                    dedup_frags=n_pub, log=True, engine_cmd=engine_cmd, timeout=180, engine_procs=engine_procs, **kw)
    assert res["engine_procs"] == engine_procs and len(res["engines"]) == engine_procs
    st = res["engine"]["stats"]
    assert st["verify_errors"] == 0 and st["corrupt"] == 0 and st["overrun"] == 0
    for k, (exp_out, exp_pub) in enumerate(exp):
        seqs, codes = res["logs"][k]
        assert seqs.tolist() == list(range(len(ps))) and codes.tolist() == exp_out
        assert [(sig, tile.split_verify_output(f)) for sig, f in res["out_frags"][k]] == \
            [(t, (p, raw)) for p, raw, t in exp_pub]
    if dedup:
        ds = res["dedup"]["stats"]
        assert res["dedup"]["exit"] == 0 and ds["overrun"] == 0 and ds["in_frags"] == n_pub
        if tiles == 1:                     # one in link: the dedup tile's order is the verify tile's
            exp_d = tile_model.dedup_model([f for _, f in res["out_frags"][0]], dseed, xproc.DEDUP_TCACHE_DEPTH)
            assert [f for _, f in res["dedup_frags"]] == exp_d
        else:
            _check_dedup_multi_link([[f for _, f in o] for o in res["out_frags"]], [f for _, f in res["dedup_frags"]])
        assert all(sig == 0 for sig, _ in res["dedup_frags"])
        assert res["dedup"]["stats"]["done_ns"] > 0
    return res, exp


def test_engine_process_pipeline_cpu(tmp_path, oracle):
    ps = _mixed_stream(600, seed=71)
    res, exp = _xproc_vs_model(tmp_path, ps, oracle, engine_cmd=CPU_ENGINE, depth=1 << 12, batch=64, inflight=3)
    assert exp[0][0].count(-2) > 10 and exp[0][0].count(-1) > 10
    assert res["engine"]["verifier"].startswith("oracle")


def test_engine_process_sandboxed_cpu(tmp_path, oracle):
    """The engine process inside its seccomp policy (--sandbox 1) once the
    tiles run: the same frag-by-frag outcomes, its result reports the
    policy; in report mode (--sandbox 2) nothing was refused."""
    ps = _mixed_stream(500, seed=77)
    res, _ = _xproc_vs_model(tmp_path, ps, oracle, engine_cmd=CPU_ENGINE, depth=1 << 12, batch=64, inflight=3,
                             sandbox=1)
    assert res["engine"]["sandbox"] == 1
    res, _ = _xproc_vs_model(tmp_path, ps, oracle, engine_cmd=CPU_ENGINE, depth=1 << 12, batch=64, inflight=3,
                             sandbox=2, dedup=False)
    assert res["engine"]["sandbox"] == 2 and res["engine"]["sandbox_refused"] == [], res["engine"]["sandbox_refused"]


def test_engine_process_two_tiles_cpu(tmp_path, oracle):
    """Two verify tiles in the engine process take the round-robin shares of
    the link (fd_verify.c:46), each into its own out link."""
    ps = _mixed_stream(800, seed=74)
    _xproc_vs_model(tmp_path, ps, oracle, tiles=2, engine_cmd=CPU_ENGINE, depth=1 << 12, batch=64, inflight=3)


def test_two_engine_processes_share_link_cpu(tmp_path, oracle):
    """Two engine processes on one shared quic -> verify link, one tile each,
    as global tiles 0 and 1 of 2 (--rr-idx 0/1 --rr-cnt 2, fd_verify.c:46):
    each equals tile_model(rr_idx, 2) frag by frag, and the sandboxed dedup
    over both out links publishes every distinct verified txn once."""
    ps = _mixed_stream(900, seed=75)
    res, exp = _xproc_vs_model(tmp_path, ps, oracle, tiles=2, engine_procs=2, engine_cmd=CPU_ENGINE, depth=1 << 12,
                               batch=64, inflight=3)
    assert [e["rr_idx"] for e in res["engines"]] == [0, 1] and all(e["rr_cnt"] == 2 for e in res["engines"])
    assert len({e["pid"] for e in res["engines"]}) == 2
    assert all(len(pub) > 100 for _, pub in exp)


def test_eight_engine_processes_cpu(tmp_path, oracle):
    """verify_tile_cnt = 8 as eight engine processes over one link (global
    tiles 0..7 of 8), the dedup over their eight out links: frag by frag
    against tile_model(k, 8) (the CPU stand-in verifier)."""
    ps = _mixed_stream(1600, seed=79)
    res, exp = _xproc_vs_model(tmp_path, ps, oracle, tiles=8, engine_procs=8, engine_cmd=CPU_ENGINE, depth=1 << 12,
                               batch=64, inflight=2)
    assert sorted(e["rr_idx"] for e in res["engines"]) == list(range(8))


def test_engine_proc_devices_and_round_robin_args():
    """--devices maps tile k to the (k % n)-th device; --rr-idx/--rr-cnt
    outside the tiles' range is refused."""
    from firedancer_amd import engine_proc
    import argparse
    a = argparse.Namespace(devices="3,5", device_rank=-1, device=0)
    assert engine_proc.tile_devices(3, a) == [3, 5, 3]
    a = argparse.Namespace(devices="", device_rank=9, device=0)
    assert engine_proc.tile_devices(2, a, ndev=8) == [1, 1]
    a = argparse.Namespace(devices="", device_rank=-1, device=2)
    assert engine_proc.tile_devices(1, a) == [2]
    assert engine_proc.round_robin_shares(2, 8, 2) == [2, 3] and engine_proc.round_robin_shares(0, 0, 3) == [0, 1, 2]
    for bad in ((1, 1, 1), (7, 8, 2), (-1, 4, 1), (0, 4, 0)):
        with pytest.raises(ValueError):
            engine_proc.round_robin_shares(*bad)


@pytest.mark.gpu
def test_engine_process_pipeline_gpu(tmp_path, oracle):
    """The deployable shape on the MI355X: the engine process's gather tile
    reads every payload where the producer process wrote it (the link's
    shared-memory region registered with its engine), verifies it on the GPU
    and writes its out frag; two tiles in the second run."""
    ps = _mixed_stream(3000, seed=72)
    res, exp = _xproc_vs_model(tmp_path, ps, oracle, depth=1 << 12, batch=512, inflight=3)
    assert exp[0][0].count(0) > 1000 and res["engine"]["device"] == 0
    assert res["engine"]["sandbox"] == 1                 # the engine policy is on by default (fdt_sandbox_engine_enter)
    _xproc_vs_model(tmp_path, ps, oracle, tiles=2, depth=1 << 12, batch=512, inflight=3, dedup=False)


@pytest.mark.gpu
def test_engine_processes_multi_device_gpu(tmp_path, oracle):
    """The multi-GPU form of the verify stage on the box's one GPU: two
    engine processes sharing the quic -> verify link (global tiles 0 and 1
    of 2), the sandboxed dedup over both out links at the reference's tcache
    depth; then one process whose two tiles are placed by --devices 0,0 (on
    an 8-GPU node: --devices 0,1,...)."""
    ps = _mixed_stream(4000, seed=76)
    res, _ = _xproc_vs_model(tmp_path, ps, oracle, tiles=2, engine_procs=2, depth=1 << 12, batch=512, inflight=3)
    assert [e["devices"] for e in res["engines"]] == [[0], [0]]
    res, _ = _xproc_vs_model(tmp_path, ps, oracle, tiles=2, engine_procs=1, proc_devices=["0,0"], depth=1 << 12,
                             batch=512, inflight=3)
    assert res["engine"]["devices"] == [0, 0]


@pytest.mark.gpu
def test_eight_engine_processes_gpu(tmp_path, oracle):
    """The node shape of BASELINE cfg5 -- verify_tile_cnt = 8, one GPU per
    tile (fd_frankendancer.c:99,131-133) -- rehearsed on the box's one GPU:
    eight engine processes, each one tile as global tile k of 8 over the same
    quic -> verify link (--rr-idx k --rr-cnt 8), each inside its seccomp
    policy, the sandboxed dedup over the eight out links at the reference's
    depth.  Every tile equals tile_model(k, 8) frag by frag; the dedup's
    output is every distinct verified txn once."""
    ps = _mixed_stream(4000, seed=78)
    res, exp = _xproc_vs_model(tmp_path, ps, oracle, tiles=8, engine_procs=8, depth=1 << 12, batch=256, inflight=2)
    assert sorted(e["rr_idx"] for e in res["engines"]) == list(range(8))
    assert all(e["rr_cnt"] == 8 and e["sandbox"] == 1 for e in res["engines"])
    assert all(len(pub) > 200 for _, pub in exp)


@pytest.mark.gpu
def test_engine_process_lapped_gpu(tmp_path, oracle):
    """The cross-process gather tile against a producer process that laps it:
    lap guard off, batches held 3 ms, a 1024-deep link fed at 1 M frags/s.
    The device's re-check drops exactly the frags the producer overwrote
    before the read; every kept frag's outcome and the published stream equal
    the model's over exactly those frags, none published torn."""
    seed = 0x1AB
    ps = _mixed_stream(20000, seed=31)
    res = xproc.run(_npz(tmp_path, ps), len(ps), tiles=1, producers=1, mode="paced", rate=1.0e6, depth=1024,
                    batch=4096, inflight=3, wait_us=3000, lap_guard=False, seed=seed, log=True, timeout=180)
    st, mux = res["engine"]["stats"], res["engine"]["mux"]
    assert st["corrupt"] == 0 and st["verify_errors"] == 0
    seqs, codes = res["logs"][0]
    assert len(seqs) + mux["overrun_polling"] + mux["overrun_reading"] == len(ps)
    lost = codes == tile.LOG_LOST
    assert int(lost.sum()) == st["lapped"] > 1000
    kept = seqs[~lost].tolist()
    exp_out, exp_pub = tile_model.verify_tile_model([ps[s] for s in kept], seed,
                                                    lambda a, t: oracle.verify_txns(a, t), seqs=kept)
    assert codes[~lost].tolist() == exp_out and len(kept) > 2000
    assert [(sig, tile.split_verify_output(f)) for sig, f in res["out_frags"][0]] == \
        [(t, (p, raw)) for p, raw, t in exp_pub]


@pytest.mark.gpu
def test_engine_process_cli_gpu(oracle, tmp_path):
    """`python -m firedancer_amd.engine_proc` as an operator starts it: joins
    links another process formatted, verifies on the GPU, prints the tiles'
    stats."""
    import json
    import subprocess
    ps = _mixed_stream(1500, seed=73)
    paths = [_shm_path(n) for n in ("qv", "vd")]
    try:
        inl = tile.Link.shm_create(paths[0], 1 << 12, 1232)
        vd = tile.Link.shm_create(paths[1], 1 << 12, tile.TPU_DCACHE_MTU,
                                  data_sz=tile.vmux_dcache_data_sz(1 << 12, 512, 3))
        for p in ps:
            inl.publish(p)
        r = subprocess.run([sys.executable, "-m", "firedancer_amd.engine_proc", "--in", paths[0], "--out", paths[1],
                            "--frags", str(len(ps)), "--batch", "512", "--inflight", "3", "--timeout", "60"],
                           capture_output=True, text=True, timeout=120, cwd=REPO)
        assert r.returncode == 0, r.stderr[-2000:]
        st = json.loads(r.stdout.strip().splitlines()[-1])["stats"]
        exp_out, exp_pub = tile_model.verify_tile_model(ps, 0x5EEDF00D, lambda a, t: oracle.verify_txns(a, t))
        assert st["published"] == exp_out.count(0) and st["verify_failed"] == exp_out.count(-1)
        assert [m["sig"] for m, _ in vd.drain()] == [t for _, _, t in exp_pub]
    finally:
        for p in paths:
            if os.path.exists(p):
                os.unlink(p)


def test_traceback_inside_engine_policy():
    """An error after the engine process entered its policy still prints a
    traceback with source lines (engine_proc caches them before entry;
    reading a source file then would be a refused open)."""
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:
        try:
            import traceback
            from firedancer_amd import engine_proc
            engine_proc._cache_source_lines()
            tile.engine_sandbox_enter()
            try:
                engine_proc.round_robin_shares(5, 2, 1)
            except ValueError:
                os.write(w, traceback.format_exc().encode())
        finally:
            os._exit(0)
    os.close(w)
    _, status = os.waitpid(pid, 0)
    tb = os.read(r, 65536).decode()
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0, status
    assert "raise ValueError" in tb and "round_robin_shares" in tb, tb


def test_driver_fds_found_by_path(tmp_path):
    """fdt_sandbox_driver_fds lists exactly the fds naming the GPU driver's
    devices: none here without them, and an fd of another file is never
    listed."""
    f = open(tmp_path / "x", "w")
    try:
        fds = tile.device_fds()
        assert f.fileno() not in fds
        for fd in fds:
            assert os.readlink(f"/proc/self/fd/{fd}") == "/dev/kfd" or \
                os.readlink(f"/proc/self/fd/{fd}").startswith("/dev/dri/")
        if not os.path.exists("/dev/kfd"):
            assert fds == []
    finally:
        f.close()
