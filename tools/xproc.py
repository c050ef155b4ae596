"""The verify stage as separate processes, the way the reference's topology
runs it (src/app/fdctl/run/topos/fd_frankendancer.c:59-60,131-133;
fd_topo_run.c:50-171): this process plays the topology launcher -- it lays
the links out in shared memory (tile.Link.shm_create, every page faulted in
first, as fd_topo allocates its workspaces up front, fd_topo.c:262-278) and
starts

  * the QUIC side: tools/quic_feed.py, one producer thread per quic -> verify
    link (a process that never touches the GPU);
  * the engine processes: python -m firedancer_amd.engine_proc, T gather-mode
    verify mux tiles over every in link, tile k publishing into its own
    verify -> dedup link -- in one process, or spread over E processes that
    share the in links, process p running global tiles p*T/E .. (p+1)*T/E-1
    of T (--rr-idx / --rr-cnt: fd_verify.c:46's seq % verify_tile_cnt);
  * optionally the dedup tile: python -m firedancer_amd.dedup_proc, a
    sandboxed child reading every verify -> dedup link;

and collects their JSON results.  Used by tests/test_engine_proc.py (parity
frag by frag against tests/tile_model.py) and tools/bench_tile.py --xproc
(the cross-process bench lines).  The launcher itself starts no HIP runtime.
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

from firedancer_amd import tile  # noqa: E402
import quic_feed  # noqa: E402

OUT_DEPTH = 1 << 14
# the dedup tile's tcache depth: the reference's signature_cache_size
# (src/app/fdctl/config/default.toml:910, wired at fd_frankendancer.c:263)
DEDUP_TCACHE_DEPTH = 4194302


def _wait_file(path, procs, timeout):
    t0 = time.monotonic()
    while not os.path.exists(path):
        for p in procs:
            if p.poll() is not None:
                out, err = p.communicate()
                raise RuntimeError(f"{p.args[:3]} exited ({p.returncode}) before {os.path.basename(path)}: "
                                   f"{err[-3000:] if err else ''}")
        if time.monotonic() - t0 > timeout:
            raise TimeoutError(f"waiting for {path}")
        time.sleep(0.002)


def _finish(p, timeout, what):
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        p.kill()
        out, err = p.communicate()
        raise RuntimeError(f"{what} timed out: {err[-3000:]}")
    if p.returncode != 0:
        raise RuntimeError(f"{what} failed ({p.returncode}): {err[-3000:]}")
    res = json.loads(out.strip().splitlines()[-1])
    if isinstance(res, dict) and err:
        res["stderr_tail"] = err[-2000:]
    return res


def run(npz, n_payloads, tiles=1, producers=1, mode="paced", rate=0.0, reps=1, depth=1 << 14, batch=16384,
        inflight=8, wait_us=200.0, batch_sig_max=0, pages="4k", cpus=None, device_rank=0, dedup=False,
        dedup_frags=0, log=False, lap_guard=True, pair=2, spread=2, seed=0x5EEDF00D, timeout=300.0,
        hw_queues=32, engine_cmd=None, engine_procs=1, proc_devices=None, dedup_depth=DEDUP_TCACHE_DEPTH,
        sandbox=None, proc_device_ranks=None):
    """One cross-process run over the payloads in `npz` (arena, offs, sizes;
    n_payloads of them).  engine_cmd: the engine process's command before
    its arguments (default: python -m firedancer_amd.engine_proc; the CPU
    tests run the same loop over their checker instead).  engine_procs: E
    engine processes over the same in links, tiles // E tiles each;
    proc_devices: per process the --devices string (default: every process
    --device-rank device_rank; proc_device_ranks: per process its
    --device-rank, the device being that % the visible devices -- a launcher
    that must not start a HIP runtime itself); sandbox: the engine processes' --sandbox
    (None: their default).  Returns {engine, engines, feed, dedup,
    wall_s, txns_per_s, ...} (engine: the processes' stats combined,
    engines: each process's own); with log=True also the tiles' per-frag
    outcomes (logs: [(seqs, codes)] per global tile) and the out links'
    frags (out_frags: per tile [(sig, payload)]) and the dedup tile's out
    frags (dedup_frags)."""
    cpus = list(cpus or [])
    E = max(1, engine_procs)
    if tiles % E:
        raise ValueError(f"{tiles} tiles over {E} engine processes")
    d = tempfile.mkdtemp(prefix="fdgpu_xp_", dir="/dev/shm")
    procs = []
    try:
        P, T = producers, tiles
        TE = T // E
        qv = [os.path.join(d, f"qv{j}") for j in range(P)]
        vd = [os.path.join(d, f"vd{k}") for k in range(T)]
        ins = [tile.Link.shm_create(p, depth, tile.TPU_MTU, pages=pages) for p in qv]
        outs = [tile.Link.shm_create(p, OUT_DEPTH, tile.TPU_DCACHE_MTU, pages=pages,
                                     data_sz=tile.vmux_dcache_data_sz(OUT_DEPTH, batch, inflight)) for p in vd]
        dp = os.path.join(d, "dp")
        if dedup:
            tile.Link.shm_create(dp, 1 << 16, tile.TPU_DCACHE_MTU)
        cnts = quic_feed.frag_counts(n_payloads, P, mode, reps)
        readies = [os.path.join(d, f"engine{e}.ready") for e in range(E)]
        pcpu, tcpu = cpus[:P], cpus[P:P + T]
        eng_cmds = []
        for e in range(E):
            c = [*(engine_cmd or [sys.executable, "-m", "firedancer_amd.engine_proc"]),
                 *sum([["--in", p] for p in qv], []), *sum([["--out", p] for p in vd[e * TE:(e + 1) * TE]], []),
                 "--frags", ",".join(map(str, cnts)), "--rr-idx", str(e * TE), "--rr-cnt", str(T),
                 "--batch", str(batch), "--inflight", str(inflight),
                 "--batch-sig-max", str(batch_sig_max), "--wait-us", str(wait_us), "--seed", hex(seed),
                 "--pair", str(pair), "--spread", str(spread), "--lap-guard", str(int(lap_guard)),
                 "--hw-queues", str(hw_queues), "--ready-file", readies[e], "--timeout", str(timeout)]
            c += (["--devices", proc_devices[e]] if proc_devices else
                  ["--device-rank", str(proc_device_ranks[e] if proc_device_ranks else device_rank)])
            if tcpu:
                c += ["--cpus", ",".join(map(str, tcpu[e * TE:(e + 1) * TE]))]
            if dedup:                        # verify -> dedup links are reliable (fd_topo): credits from the dedup's fseq
                c += ["--out-flow-control", "1"]
            if sandbox is not None:
                c += ["--sandbox", str(sandbox)]
            if log:
                c += ["--log", os.path.join(d, f"log{e}.npz")]
            eng_cmds.append(c)
        feed_cmd = [sys.executable, os.path.join(REPO, "tools", "quic_feed.py"), *sum([["--link", p] for p in qv], []),
                    "--npz", npz, "--mode", mode, "--rate", str(rate), "--reps", str(reps)]
        if pcpu:
            feed_cmd += ["--cpus", ",".join(map(str, pcpu))]
        popen = dict(stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=REPO)
        feed = None
        if mode == "prefill":                    # every frag published before the tiles start
            feed = _finish(subprocess.Popen(feed_cmd, **popen), timeout, "quic_feed")
        engs = [subprocess.Popen(c, **popen) for c in eng_cmds]
        procs += engs
        for r in readies:
            _wait_file(r, engs, timeout)
        dd = None
        if dedup:
            dd_cmd = [sys.executable, "-m", "firedancer_amd.dedup_proc", *sum([["--in", p] for p in vd], []),
                      "--out", dp, "--frags", str(dedup_frags or (1 << 62)), "--idle-s", "3", "--reliable", "1",
                      "--tcache-depth", str(dedup_depth)]
            if len(cpus) > P + T:
                dd_cmd += ["--cpu", str(cpus[P + T])]
            dd = subprocess.Popen(dd_cmd, **popen)
            procs.append(dd)
        if mode != "prefill":
            fp = subprocess.Popen(feed_cmd + sum([["--wait-file", r] for r in readies], []), **popen)
            procs.append(fp)
            feed = _finish(fp, timeout, "quic_feed")
        ers = [_finish(p, timeout, "engine_proc") for p in engs]
        er = combine_engine_results(ers)
        res = {"engine": er, "engines": ers, "feed": feed}
        if dd is not None:
            res["dedup"] = _finish(dd, 60, "dedup_proc")
        t0 = er["t_start"] if mode == "prefill" else max(er["t_start"], feed["t_start"])
        # with the dedup in the loop the run ends when its last frag has gone through it
        t_end = max(er["t_done"], res["dedup"]["stats"]["done_ns"] * 1e-9) if dd is not None else er["t_done"]
        wall = t_end - t0
        n_total = sum(cnts)
        res.update({"wall_s": round(wall, 6), "txns": n_total, "txns_per_s": round(n_total / wall, 1),
                    "frag_counts": cnts, "pages": pages, "link_depth": depth, "engine_procs": E,
                    "in_huge_bytes": er.get("in_huge_bytes"), "feed_huge_bytes": feed.get("huge_bytes")})
        if log:
            res["logs"] = []
            for e in range(E):
                z = np.load(os.path.join(d, f"log{e}.npz"))
                res["logs"] += [(z[f"seq{k}"], z[f"code{k}"]) for k in range(TE)]
            res["out_frags"] = [[(m["sig"], bytes(f)) for m, f in ln.drain()] for ln in outs]
            if dedup:
                res["dedup_frags"] = [(m["sig"], bytes(f)) for m, f in tile.Link.shm_join(dp).drain()]
        del ins, outs
        return res
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        shutil.rmtree(d, ignore_errors=True)


def combine_engine_results(ers):
    """The engine processes' results as one: counters summed (extremes as
    extremes), started at the first process's start, done at the last's."""
    if len(ers) == 1:
        return ers[0]
    out = dict(ers[0])
    st = {}
    for k in ers[0]["stats"]:
        xs = [r["stats"][k] for r in ers]
        st[k] = max(xs) if k.endswith(("_max", "_max_ns")) else min(xs) if k.endswith(("_min", "_min_ns")) else sum(xs)
    out.update({"stats": st, "mux": {k: sum(r["mux"][k] for r in ers) for k in ers[0]["mux"]},
                "tiles": sum(r["tiles"] for r in ers), "t_start": min(r["t_start"] for r in ers),
                "t_done": max(r["t_done"] for r in ers), "pid": [r["pid"] for r in ers],
                "per_tile": sum((r["per_tile"] for r in ers), []), "final": sum((r["final"] for r in ers), []),
                "devices": sum((r.get("devices") or [r.get("device")] for r in ers), [])})
    lat = [r["batch_latency_ms"] for r in ers]
    out["batch_latency_ms"] = {"p50": max((x["p50"] for x in lat if x["p50"] is not None), default=None),
                               "p99": max((x["p99"] for x in lat if x["p99"] is not None), default=None),
                               "n": sum(x["n"] for x in lat), "note": "worst process's percentile"}
    return out


def save_payloads(ps, path):
    """payload list -> the npz quic_feed.py reads"""
    arena, offs, sizes = tile_pack(ps)
    np.savez(path, arena=arena, offs=offs, sizes=sizes)
    return path


def tile_pack(ps):
    from firedancer_amd import workload
    return workload.pack_payloads(ps)
