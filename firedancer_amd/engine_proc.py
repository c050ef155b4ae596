"""The verify stage's GPU side as its own process (SURVEY.md §8(f) row 1,
"seccomp or separate engine process").

The reference runs every tile as its own process: the verify tiles join the
quic -> verify links that the QUIC tiles' processes publish into, in
workspaces the topology allocates up front (src/app/fdctl/run/topos/
fd_frankendancer.c:59-60,131-133, src/disco/topo/fd_topo_run.c:50-171,
src/app/fdctl/run/tiles/fd_verify.c:150-207), and after privileged init
only write/fsync remain (verify.seccomppolicy:1-19, entered at
fd_topo_run.c:96-103).  HIP needs ioctls on /dev/kfd for every submission,
so the batched verify tile runs here, unsandboxed, in a process of its own
-- the wiredancer arrangement (src/wiredancer/c/wd_f1.h:71-112) -- and joins
the links by path (tile.Link.shm_join / fdt_link_join).  Tiles that only
touch links (dedup, and any other consumer) keep the reference's sandbox
(firedancer_amd/dedup_proc.py).

The tile this process runs is the measured one: T verify mux tiles
(fdgpu_vmux on fdt_mux_run, the fd_verify.c:232-246 callbacks) in the
gather mode (gpu_parse 2): the device reads each payload where the producer
process wrote it (the in links' regions are registered with the engines),
parses, verifies, tags it and writes the out frag into the out link's
dcache; tile k publishes into out link k.

A node's verify stage spans its GPUs the way the reference spans cores:
verify_tile_cnt tiles each read every quic -> verify link and take the
round-robin share `seq % verify_tile_cnt == tile index` of it
(src/app/fdctl/run/topos/fd_frankendancer.c:99,131-133,
src/app/fdctl/run/tiles/fd_verify.c:36-47).  Here tile k of this process is
global tile rr_idx + k of rr_cnt (--rr-idx / --rr-cnt), and its engine sits
on devices[k % len(devices)] (--devices): one process per GPU (N processes,
--rr-idx p*T --rr-cnt N*T, --devices p) or one process over several GPUs
(--devices 0,1,...) share the same links, with no collective between them.

    python -m firedancer_amd.engine_proc --in /dev/shm/quic_verify_0 \\
        [--in ...] --out /dev/shm/verify_dedup_0 [--out ...] --frags N[,N...] \\
        [--devices 0,1] [--rr-idx 0 --rr-cnt 2]

runs until every frag the producers will publish (--frags, per in link) has
its outcome -- or, once the producers are done, until the tiles sit idle --
and prints the tiles' stats as one JSON line (--result: also into a file).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

from . import tile

# HIP hardware queues of this process (set before the runtime starts): each
# tile engine owns `inflight` slot streams; two busy streams sharing a queue
# serialise
DEFAULT_HW_QUEUES = 32
# the engine seccomp policy (fdt_sandbox_engine_enter) once the tiles run
DEFAULT_SANDBOX = 1


def warm_engines(engines, inflight, out_bytes=0, batch=64):
    """A full-size batch through every ring slot of every engine before any
    timed run: a HIP stream's first submission creates its hardware queue
    (milliseconds), and a slot sizes its buffers on first use to the batch
    it carries -- both would otherwise land inside the run.  out_bytes > 0:
    the gathered path's slot buffers too (fdgpu_submit_frags_io)."""
    from . import workload
    from .ed25519 import FRAG_IO_DTYPE
    from . import _lib
    a, t, _ = workload.cfg1(64, seed=7)
    ps = workload.payloads(a, t)
    ps = [ps[k % len(ps)] for k in range(batch)]
    a, t, _ = workload.cfg1(batch, seed=7)
    pa, po, psz = workload.pack_payloads(ps)
    fx = np.zeros(len(ps), dtype=tile.FRAG_EX_DTYPE)
    fx["off"], fx["sz"] = po, psz
    tr = 0
    for k, p in enumerate(ps):
        fp, _ = tile.txn_peek(p)
        fx[k]["tr_off"], fx[k]["tr_cap"] = tr, fp
        tr += (fp + 3) & ~3
    for e in engines:
        tks = [e.submit(a, t) for _ in range(inflight)]
        for tk in tks:
            e.poll(tk, blocking=True)
        tks = [e.submit_frags(pa, fx, tr) for _ in range(inflight)]
        for tk in tks:
            e.poll_frags(tk, blocking=True)
    if not out_bytes:
        return
    L = _lib.lib()
    src = tile._page_buf(len(ps) * 1280 + 4096)
    out = tile._page_buf(out_bytes + 4096)
    fio = np.zeros(len(ps), dtype=FRAG_IO_DTYPE)
    o = 0
    for k, p in enumerate(ps):
        src[k * 1280:k * 1280 + len(p)] = np.frombuffer(p, dtype=np.uint8)
        cap = L.fdgpu_frag_out_cap(len(p))
        fio[k] = (src.ctypes.data + k * 1280, len(p), o, cap, 0, 0)
        o += (cap + 63) // 64 * 64
    for e in engines:
        e.host_register(src)
        e.host_register(out)
        tks = [e.submit_frags_io(fio, out, out_bytes, 1) for _ in range(inflight)]
        for tk in tks:
            e.poll_frags_io(tk, blocking=True)
        e.host_unregister(src)
        e.host_unregister(out)


def open_engines(n, device, batch, inflight, pair=2, spread=2, gather=True):
    """n tile engines as the tile lines open them (one per tile; the comb
    table is shared per device), every slot reserved and warmed.  device: one
    HIP device for all, or a list (engine k on device[k % len])."""
    from . import VerifyEngine
    frag_bytes = (tile.TPU_DCACHE_MTU + 63) // 64 * 64
    devs = list(device) if isinstance(device, (list, tuple)) else [device]
    es = []
    for k in range(n):
        e = VerifyEngine(devs[k % len(devs)], max_txn=batch, max_sig=batch * 12, max_arena=batch * frag_bytes,
                         ring_depth=inflight, pair=pair == 1, pair_auto=pair == 2, spread=spread == 1,
                         spread_auto=spread == 2)
        e.reserve()
        es.append(e)
    warm_engines(es, inflight, out_bytes=batch * frag_bytes if gather else 0, batch=batch)
    return es


def _producers_done(ins, frag_cnts):
    """Every in link's producer has published its last frag (that seq's line
    holds it, or a later one: lapped past)."""
    for ln, n in zip(ins, frag_cnts):
        if n and ln.poll(ln.seq0 + n - 1)[0] == 0:          # 0: not yet published
            return False
    return True


def _cache_source_lines():
    """Read every loaded module's source into linecache now: inside the
    engine policy a traceback could not open them (open is refused, and in
    enforce mode fatal), so an error after entry would die without one.  The
    cache is not re-validated afterwards (that stats each file by path, which
    the policy refuses too; the sources do not change under a running
    process)."""
    import linecache
    for m in list(sys.modules.values()):
        f = getattr(m, "__file__", None)
        if f and f.endswith(".py"):
            linecache.getlines(f)
    linecache.checkcache = lambda filename=None: None


def round_robin_shares(rr_idx, rr_cnt, T):
    """The global round-robin index of each of this process's T tiles
    (fd_verify.c:46: tile i of verify_tile_cnt takes seq % cnt == i):
    rr_idx .. rr_idx+T-1 of rr_cnt (0: T)."""
    rr_cnt = rr_cnt or T
    if T < 1 or rr_idx < 0 or rr_idx + T > rr_cnt:
        raise ValueError(f"round robin: {T} tiles from index {rr_idx} of {rr_cnt}")
    return list(range(rr_idx, rr_idx + T))


def serve(in_paths, out_paths, verifiers, frag_cnts, timeout_s=120.0, idle_s=0.02, cpus=None, ready_file=None,
          log_max=0, on_start=None, rr_idx=0, rr_cnt=0, sandbox=0, **tile_kw):
    """Join the links, run one gather-mode verify mux tile per out link
    (tile k: round-robin share rr_idx + k of rr_cnt (0: of this process's
    tiles) of every in link, verifiers[k], out link k)
    until the outcome of every frag is final -- or, when frags were lost to
    the producers, until they are done and the tiles sit idle for idle_s --
    then return {stats, mux, per-tile stats, latencies, times}.  cpus: tile
    k's thread is pinned to cpus[k].  ready_file: created once the tiles are
    polling (a producer process waits for it).  sandbox: 1 -- from then on
    the process runs inside the engine policy (tile.engine_sandbox_enter:
    no open, socket, exec or fork; ioctl only on the GPU driver's fds held
    now), 2 -- the same policy in report mode (a refused call fails and is
    listed in the result instead of killing the process), 0 -- none."""
    ins = [tile.Link.shm_join(p) for p in in_paths]
    outs = [tile.Link.shm_join(p) for p in out_paths]
    # huge-page accounting reads /proc/self/smaps: before the sandbox, and
    # before the timed region (tens of ms on a 2 GB link of 4 KB pages)
    in_huge = [ln.huge_bytes() for ln in ins]
    T = len(outs)
    rr = round_robin_shares(rr_idx, rr_cnt, T)
    frag_cnts = list(frag_cnts)
    n_total = sum(frag_cnts)
    tile_kw.setdefault("gpu_parse", 2)
    vms = [tile.VerifyMuxTile(ins, outs[k], verifiers[k], round_robin_idx=rr[k], round_robin_cnt=rr_cnt or T,
                              log_max=log_max, **tile_kw) for k in range(T)]
    try:
        t_start = time.monotonic()
        for k, vm in enumerate(vms):
            vm.start(cpu=cpus[k % len(cpus)] if cpus else None)
        if on_start:
            on_start()
        if ready_file:
            with open(ready_file + ".tmp", "w") as f:
                f.write(str(os.getpid()))
            os.rename(ready_file + ".tmp", ready_file)
        if sandbox:                    # engines open, warmed, registered; tiles running (fd_topo_run.c:96-103)
            _cache_source_lines()
            tile.engine_sandbox_enter(report=sandbox == 2)
        idle_since, last = None, -1
        while any(vm.final_cnt() < n_total for vm in vms):
            now = time.monotonic()
            if now - t_start > timeout_s:
                raise TimeoutError(f"engine process: {[vm.final_cnt() for vm in vms]} of {n_total} frags final")
            for vm in vms:
                if tile.lib().fdgpu_vmux_error(vm._t):
                    raise RuntimeError(f"verify mux tile: verifier error {tile.lib().fdgpu_vmux_error(vm._t)}")
            cur = sum(vm.final_cnt() for vm in vms)
            if cur != last or not all(vm.idle() for vm in vms) or not _producers_done(ins, frag_cnts):
                idle_since, last = now, cur
            elif now - idle_since > idle_s:
                break
            time.sleep(0.0002)
        t_done = time.monotonic() if idle_since is None or all(vm.final_cnt() >= n_total for vm in vms) \
            else idle_since
        for vm in vms:
            vm.stop()
        per = [vm.stats() for vm in vms]
        mux = [vm.mux_stats() for vm in vms]
        lat = np.concatenate([vm.latencies_ns() for vm in vms]) / 1e6 if vms else np.zeros(0)
        agg = {k: int(sum(s[k] for s in per)) for k in per[0]}
        for k in agg:                       # extremes combine as extremes, not sums
            if k.endswith("_max") or k.endswith("_max_ns"):
                agg[k] = max(s[k] for s in per)
            elif k.endswith("_min") or k.endswith("_min_ns"):
                agg[k] = min(s[k] for s in per)
        magg = {k: int(sum(m[k] for m in mux)) for k in mux[0]}
        agg["overrun_polling"], agg["overrun_reading"] = magg["overrun_polling"], magg["overrun_reading"]
        agg["overrun"] = agg["lapped"] + agg["overrun_polling"] + agg["overrun_reading"]
        res = {"pid": os.getpid(), "tiles": T, "rr_idx": rr_idx, "rr_cnt": rr_cnt or T, "in_links": len(ins), "frags": n_total,
               "t_start": t_start, "t_done": t_done, "stats": agg, "mux": magg, "per_tile": per,
               "final": [int(vm.final_cnt()) for vm in vms],
               "batch_latency_ms": {"p50": round(float(np.percentile(lat, 50)), 3) if len(lat) else None,
                                    "p99": round(float(np.percentile(lat, 99)), 3) if len(lat) else None,
                                    "n": int(len(lat))},
               "in_huge_bytes": in_huge}
        if log_max:
            res["logs"] = [vm.log() for vm in vms]
        res["sandbox"] = sandbox
        if sandbox == 2:
            res["sandbox_refused_calls"], res["sandbox_refused"] = tile.engine_sandbox_report()
        return res
    finally:
        for vm in vms:
            vm.close()
        if sandbox == 2:                 # bring-up: what the policy refused, whatever the outcome
            sys.stderr.write(f"engine_proc: sandbox refused {tile.engine_sandbox_report()}\n")


def tile_devices(T, a, ndev=None):
    """The HIP device of each of this process's T tiles: --devices (tile k on
    the (k % n)-th), else --device-rank % the visible devices, else --device."""
    if a.devices:
        devs = [int(x) for x in a.devices.split(",") if x.strip()]
    elif a.device_rank >= 0:
        if ndev is None:
            from . import _lib
            ndev = _lib.lib().fdgpu_device_count()
        if ndev < 1:
            raise SystemExit("engine_proc: no HIP device visible")
        devs = [a.device_rank % ndev]
    else:
        devs = [a.device]
    return [devs[k % len(devs)] for k in range(T)]


def gpu_verifiers(T, a):
    """The product's verifiers: one GPU engine per tile (its own ring slots,
    the device's shared comb table) on the tile's device, opened, reserved
    and warmed."""
    devs = tile_devices(T, a)
    engines = open_engines(T, devs, a.batch, a.inflight, pair=a.pair, spread=a.spread, gather=a.gpu_parse == 2)
    vers = [tile.EngineVerifier([engines[k]]) for k in range(T)]

    def close():
        for v in vers:
            v.close()
        for e in engines:
            e.close()
    return vers, close, {"device": devs[0], "devices": devs}


def main(argv=None, make_verifiers=gpu_verifiers):
    """The command line above.  make_verifiers(T, args) -> (verifiers, close,
    info): the GPU engines in the product; a test substitutes its checker."""
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--in", dest="in_paths", action="append", required=True, help="a quic -> verify link (repeat)")
    ap.add_argument("--out", dest="out_paths", action="append", required=True,
                    help="a verify -> dedup link, one verify tile each (repeat)")
    ap.add_argument("--frags", required=True, help="frags the producer publishes on each in link (N or N1,N2,...)")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--device-rank", type=int, default=-1, help="device = this rank %% the visible devices")
    ap.add_argument("--devices", default="", help="','-separated HIP devices: tile k's engine on the (k %% n)-th "
                                                  "(overrides --device / --device-rank)")
    ap.add_argument("--rr-idx", type=int, default=0,
                    help="global round-robin index of this process's first tile (tile k takes share rr_idx + k)")
    ap.add_argument("--rr-cnt", type=int, default=0,
                    help="verify tiles over every engine process reading these in links (0: this process's)")
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--inflight", type=int, default=8)
    ap.add_argument("--batch-sig-max", type=int, default=0)
    ap.add_argument("--wait-us", type=float, default=200.0)
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EEDF00D)
    ap.add_argument("--gpu-parse", type=int, default=2, help="2: the gather mode (the default and measured tile)")
    ap.add_argument("--pair", type=int, default=2)
    ap.add_argument("--spread", type=int, default=2)
    ap.add_argument("--lap-guard", type=int, default=1)
    ap.add_argument("--cpus", default="", help="','-separated CPUs, tile k pinned to the k-th")
    ap.add_argument("--hw-queues", type=int, default=DEFAULT_HW_QUEUES)
    ap.add_argument("--ready-file", default="", help="created once the tiles are polling")
    ap.add_argument("--result", default="", help="also write the JSON result here")
    ap.add_argument("--log", default="", help="write every frag's outcome (seq, code per tile) to this .npz")
    ap.add_argument("--timeout", type=float, default=120.0)
    ap.add_argument("--idle-ms", type=float, default=20.0)
    ap.add_argument("--sandbox", type=int, default=DEFAULT_SANDBOX,
                    help="1: enter the engine seccomp policy once the tiles run (no open/socket/exec/fork; ioctl "
                         "only on the GPU driver's fds); 2: the same, refused calls reported instead of fatal; 0: none")
    ap.add_argument("--out-flow-control", type=int, default=0,
                    help="1: each tile takes its out link's credits from the link's fseq -- a reliable consumer "
                         "(the dedup process, dedup_proc --reliable 1) holds the tile back instead of being lapped")
    a = ap.parse_args(argv)
    cnts = [int(x) for x in a.frags.split(",")]
    if len(cnts) == 1 and len(a.in_paths) > 1:
        cnts = cnts * len(a.in_paths)
    if len(cnts) != len(a.in_paths):
        raise SystemExit("--frags: one count, or one per --in")
    T = len(a.out_paths)
    vers, close, info = make_verifiers(T, a)
    guard = {} if a.lap_guard else dict(lap_span_max=tile.LAP_OFF, lap_margin=tile.LAP_OFF)
    # inside the sandbox nothing can be opened: the output files are opened
    # now, and what writing them imports is imported now
    res_f = open(a.result, "w") if a.result else None
    log_f = open(a.log, "wb") if a.log else None
    if log_f:
        import zipfile  # noqa: F401  (np.savez imports it on first use)
    try:
        res = serve(a.in_paths, a.out_paths, vers, cnts, timeout_s=a.timeout, idle_s=a.idle_ms / 1e3,
                    cpus=[int(x) for x in a.cpus.split(",") if x] or None, ready_file=a.ready_file or None,
                    log_max=(sum(cnts) + 16) if a.log else 0, hashmap_seed=a.seed, batch_txn_max=a.batch,
                    inflight_max=a.inflight, batch_wait_us=a.wait_us, batch_sig_max=a.batch_sig_max,
                    gpu_parse=a.gpu_parse, flow_control=bool(a.out_flow_control), rr_idx=a.rr_idx, rr_cnt=a.rr_cnt,
                    sandbox=a.sandbox, **guard)
    finally:
        close()
    res.update(info)
    if log_f:
        logs = res.pop("logs")
        np.savez(log_f, **{f"seq{k}": s for k, (s, _) in enumerate(logs)},
                 **{f"code{k}": cd for k, (_, cd) in enumerate(logs)})
        log_f.close()
    line = json.dumps(res)
    if res_f:
        res_f.write(line + "\n")
        res_f.close()
    print(line, flush=True)
    return 0


if __name__ == "__main__":
    # the hardware-queue budget must be in the environment before HIP starts
    for _i, _a in enumerate(sys.argv):
        if _a.startswith("--hw-queues"):
            _v = _a.split("=", 1)[1] if "=" in _a else sys.argv[_i + 1]
            if int(_v):
                os.environ["GPU_MAX_HW_QUEUES"] = _v
            break
    else:
        os.environ.setdefault("GPU_MAX_HW_QUEUES", str(DEFAULT_HW_QUEUES))
    sys.exit(main())
