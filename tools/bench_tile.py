"""Config-5 line-rate bench (BASELINE.json configs[4]):
tango-framed cfg3 transactions (1-12 signatures, msgs up to the MTU) are
published by a producer thread into the quic->verify link; T verify tiles
(one host thread each, round-robin shares of the stream as in
fd_verify.c:46) batch them onto G GPU engines, resolve tcache/dedup in order
and publish the verify->dedup frags.  Reports end-to-end transactions/s and
signatures/s (producer start -> last frag resolved), per-batch latency
(first frag ingested -> batch published) and per-tile counters.

    python tools/bench_tile.py --gpus 1 --tiles 1 --txns 200000
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
# HIP hardware queues (see bench.py HW_QUEUES); --hw-queues overrides, 0 keeps the environment's
for i, a in enumerate(sys.argv):
    if a.startswith("--hw-queues"):
        v = a.split("=", 1)[1] if "=" in a else sys.argv[i + 1]
        if int(v):
            os.environ["GPU_MAX_HW_QUEUES"] = v
        break
else:
    os.environ["GPU_MAX_HW_QUEUES"] = "32"

import firedancer_amd as fa  # noqa: E402
from firedancer_amd import tile, workload  # noqa: E402


def make_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=200_000)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--tiles", type=int, default=0, help="verify tile threads (default: one per GPU)")
    ap.add_argument("--rate", type=float, default=0.0, help="producer frags/s (0: as fast as possible)")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--inflight", type=int, default=3)
    ap.add_argument("--wait-us", type=float, default=200.0)
    ap.add_argument("--depth-lg", type=int, default=19, help="log2 of the quic->verify mcache depth")
    ap.add_argument("--multi", type=int, default=1, help="1: cfg3 multi-sig txns, 0: cfg1 single-sig")
    ap.add_argument("--mux", type=int, default=0,
                    help="1: the verify tile as mux callbacks (fdgpu_vmux on fdt_mux_run; frags copied once into "
                         "the registered out dcache and DMA'd from there), 0: the step-loop tile (fdgpu_vtile)")
    ap.add_argument("--gpu-parse", type=int, default=2,
                    help="(mux tile) 2: the GPU reads the payloads where they lie and writes the out frags "
                         "(fdgpu_submit_frags_io); 1: fd_txn_parse on the GPU (fdgpu_submit_frags); 0: on the "
                         "tile's core")
    ap.add_argument("--producers", type=int, default=1,
                    help="(mux tile) quic->verify links, one producer thread each; every verify tile reads all of "
                         "them round robin (fd_frankendancer.c: all verify tiles read all QUIC tiles)")
    ap.add_argument("--producers-same-as-tiles", type=int, default=0,
                    help="1: as many quic links (producers) as verify tiles in every run")
    ap.add_argument("--pin", type=int, default=1,
                    help="1: producer and each tile thread pinned to its own physical core (workload.physical_cpus)")
    ap.add_argument("--cpu-offset", type=int, default=0,
                    help="skip this many of workload.physical_cpus() before pinning (CPU 0 takes interrupts)")
    ap.add_argument("--reps", type=int, default=1, help="repeat every run of the sweep")
    ap.add_argument("--hw-queues", type=int, default=32,
                    help="GPU_MAX_HW_QUEUES for this process (applied before HIP starts; 0: the environment's)")
    ap.add_argument("--out", default="")
    ap.add_argument("--sweep", default="",
                    help="';'-separated runs of 'tiles,batch,inflight,rate[,producers[,batch_sig_max[,engine_procs"
                         "[,dedup]]]]' over the same txns (batch_sig_max 0: --batch-sig-max; engine_procs and dedup: "
                         "xproc runs, 0 = the flags')")
    ap.add_argument("--payload-npz", default="",
                    help="take the frags from this .npz (arena, offs, sizes, modes, n_sig: bench.py's tile lines) "
                         "instead of generating --txns")
    ap.add_argument("--depth-lg-paced", type=int, default=0,
                    help="log2 of the link depth for paced runs (rate > 0); 0: --depth-lg")
    ap.add_argument("--warm-runs", type=int, default=0,
                    help="untimed runs of the first sweep setting before the measured ones (in-process shapes)")
    ap.add_argument("--prefill-reps", type=int, default=1,
                    help="capacity runs (rate < 0): each link carries the frag stream this many times over")
    ap.add_argument("--paced-reps", type=int, default=1,
                    help="paced runs publish the frag stream this many times over (a long stream on a shallow "
                         "link: the producers can lap the tiles)")
    ap.add_argument("--lap-guard", type=int, default=1, help="gather tile: 1 the lap guard on (default), 0 off")
    ap.add_argument("--batch-sig-max", type=int, default=0,
                    help="(mux tile) signatures per batch, counted by the frag-size bound the tile sees "
                         "(0: 12 x batch): bounds the GPU work, and the latency, of multi-signature batches")
    ap.add_argument("--pair", type=int, default=0,
                    help="(mux tile) verify kernel: 0 one lane per signature, 1 two lanes (FDGPU_FLAG_PAIR), "
                         "2 two lanes while the engine is otherwise idle (FDGPU_FLAG_PAIR_AUTO)")
    ap.add_argument("--spread", type=int, default=0,
                    help="(mux tile) verify blocks: 0 as the GPU packs them, 1 one per CU (FDGPU_FLAG_SPREAD), "
                         "2 one per CU while the engine's batches fit the chip that way (FDGPU_FLAG_SPREAD_AUTO)")
    ap.add_argument("--merge", type=int, default=0,
                    help="(mux tile) 1: FDGPU_FLAG_MERGE engines -- the verifies of an engine's batches ready at "
                         "once run as one launch")
    ap.add_argument("--tiles-per-engine", type=int, default=1,
                    help="verify tiles sharing one engine (its ring slots): a process's HIP streams are hardware "
                         "queues, and past ~20 of them the GPU's scheduler time-slices the queues")
    ap.add_argument("--reserve", type=int, default=1,
                    help="1: size every engine slot for max_sig before timing (fdgpu_engine_reserve)")
    ap.add_argument("--cpu-list", default="", help="','-separated CPUs to pin producers and tiles to, in order")
    ap.add_argument("--device", type=int, default=-1, help="the GPU every tile's engine uses (-1: tile k on k %% gpus)")
    ap.add_argument("--xproc", type=int, default=0,
                    help="1: the deployable shape -- producers in a process of their own (tools/quic_feed.py), the "
                         "gather-mode mux tiles in the engine process (python -m firedancer_amd.engine_proc), links "
                         "in shared memory faulted in before the run (tools/xproc.py); this process opens no engine")
    ap.add_argument("--pages", default="4k", help="(xproc) link memory: 4k, shm-thp or hugetlb (tile.PAGES)")
    ap.add_argument("--link-pages", default="",
                    help="(in-process mux) link memory faulted in before the run: 4k or thp (anonymous 2 MB "
                         "pages); empty: numpy pages faulted in by their first use")
    ap.add_argument("--dedup", type=int, default=0, help="(xproc) 1: a sandboxed dedup process reads the out links")
    ap.add_argument("--dedup-depth", type=int, default=4194302,
                    help="(xproc) the dedup tile's tcache depth (the reference's signature_cache_size)")
    ap.add_argument("--engine-procs", type=int, default=1,
                    help="(xproc) engine processes sharing the quic -> verify links, tiles / E tiles each (global "
                         "round-robin shares, engine_proc --rr-idx / --rr-cnt)")
    ap.add_argument("--device-rank", type=int, default=-1,
                    help="(bench.py's ranks) the GPU every tile's engine uses is this rank %% the visible devices: the "
                         "child counts them, so its parent rank starts no HIP runtime of its own before the tiles run")
    return ap


def main():
    args = make_parser().parse_args()
    if args.device_rank >= 0 and not args.xproc:
        from firedancer_amd import _lib
        ndev = _lib.lib().fdgpu_device_count()
        if ndev < 1:
            raise SystemExit("bench_tile: no HIP device visible")
        args.device = args.device_rank % ndev
    t0 = time.time()
    if args.payload_npz:
        z = np.load(args.payload_npz)
        arena, offs, sizes, modes, n_sig = z["arena"], z["offs"], z["sizes"], z["modes"], int(z["n_sig"])
        ps = [arena[o:o + n].tobytes() for o, n in zip(offs.tolist(), sizes.tolist())]
    else:
        gen = workload.cfg3 if args.multi else workload.cfg1
        a, t, modes = gen(args.txns, seed=0x5EED0005)
        ps = workload.payloads(a, t)
        arena, offs, sizes = workload.pack_payloads(ps)
        n_sig = int(t["sig_cnt"].sum())
        del a, t
    if args.xproc and not args.payload_npz:
        import tempfile
        _NPZ["path"] = os.path.join(tempfile.mkdtemp(prefix="fdgpu_bt_"), "frags.npz")
        np.savez(_NPZ["path"], arena=arena, offs=offs, sizes=sizes)
    print(f"[bench_tile] {len(ps)} txns / {n_sig} sigs ready in {time.time() - t0:.1f}s", flush=True)
    cpus = [int(x) for x in args.cpu_list.split(",") if x] or None
    depth_lg = args.depth_lg

    runs = [tuple(float(x) for x in r.split(",")) for r in args.sweep.split(";") if r] or \
        [(args.tiles or args.gpus, args.batch, args.inflight, args.rate)]
    runs = [r for r in runs for _ in range(max(1, args.reps))]
    ok = True
    lines = []
    prods0, sig_max0 = args.producers, args.batch_sig_max
    # untimed warm-up runs of the first setting: the first run of a fresh process ran slow (two tiles
    # at capacity 46 M against 69-70 M next, with the tiles' own counters equal: the time went outside
    # them; one tile paced at 24 M lost 32 K frags there, none after)
    for _ in range(max(0, args.warm_runs)):
        run = runs[0]
        args.producers = int(run[4]) if len(run) > 4 else int(run[0]) if args.producers_same_as_tiles else prods0
        args.batch_sig_max = int(run[5]) if len(run) > 5 and run[5] > 0 else sig_max0
        args.depth_lg = args.depth_lg_paced if run[3] > 0 and args.depth_lg_paced else depth_lg
        if args.xproc:
            break
        if args.mux:
            run_once_mux(args, ps, arena, offs, sizes, n_sig, modes, int(run[0]), int(run[1]), int(run[2]), run[3],
                         cpus=cpus, device=args.device if args.device >= 0 else None)
        else:
            run_once(args, ps, arena, offs, sizes, n_sig, modes, int(run[0]), int(run[1]), int(run[2]), run[3])
    procs0, dedup0 = args.engine_procs, args.dedup
    for run in runs:
        tiles_n, batch, inflight, rate = run[:4]
        # a fifth field sets the run's quic links (producers), a sixth its batches' signature cap, a seventh
        # and eighth (xproc) its engine processes and whether the sandboxed dedup reads the out links
        args.producers = int(run[4]) if len(run) > 4 else int(tiles_n) if args.producers_same_as_tiles else prods0
        args.batch_sig_max = int(run[5]) if len(run) > 5 and run[5] > 0 else sig_max0
        args.engine_procs = int(run[6]) if len(run) > 6 and run[6] > 0 else procs0
        args.dedup = int(run[7]) if len(run) > 7 else dedup0
        args.depth_lg = args.depth_lg_paced if rate > 0 and args.depth_lg_paced else depth_lg
        if args.xproc:
            res = run_once_xproc(args, n_sig, modes, len(ps), int(tiles_n), int(batch), int(inflight), rate,
                                 cpus=cpus)
        elif args.mux:
            res = run_once_mux(args, ps, arena, offs, sizes, n_sig, modes, int(tiles_n), int(batch), int(inflight),
                               rate, cpus=cpus, device=args.device if args.device >= 0 else None)
        else:
            res = run_once(args, ps, arena, offs, sizes, n_sig, modes, int(tiles_n), int(batch), int(inflight), rate)
        line = json.dumps(res)
        print(line, flush=True)
        lines.append(line)
        ok &= res["published_ok"] and res["counters"]["overrun"] == 0 and res.get("dedup_ok", True)
    if args.out:
        with open(args.out, "w") as f:
            f.write("\n".join(lines) + "\n")
    for pool in _POOL.values():
        for e in pool:
            e.close()
    return 0 if ok else 1


def run_once_xproc(args, n_sig, modes, n_payloads, tiles_n, batch, inflight, rate, cpus=None):
    """One run of the cross-process shape (tools/xproc.py): links in shared
    memory, producers in their own process, the gather-mode mux tiles in the
    engine process; the same result keys as run_once_mux."""
    import xproc
    npz = args.payload_npz or _NPZ["path"]
    P = max(1, args.producers)
    prefill = rate < 0
    reps = 1 if prefill else max(1, getattr(args, "paced_reps", 1))
    cpus = cpus or workload.physical_cpus()[getattr(args, "cpu_offset", 0):] or workload.physical_cpus()
    dev_rank = args.device_rank if args.device_rank >= 0 else max(args.device, 0)
    E = max(1, getattr(args, "engine_procs", 1))
    r = xproc.run(npz, n_payloads, tiles=tiles_n, producers=P, mode="prefill" if prefill else "paced",
                  rate=0.0 if prefill else rate, reps=reps, depth=1 << args.depth_lg, batch=batch, inflight=inflight,
                  wait_us=args.wait_us, batch_sig_max=getattr(args, "batch_sig_max", 0), pages=args.pages,
                  cpus=cpus[:P + tiles_n + 1], device_rank=dev_rank, dedup=bool(args.dedup),
                  lap_guard=bool(args.lap_guard), pair=args.pair, spread=args.spread, hw_queues=args.hw_queues,
                  dedup_frags=int((modes == 0).sum()) * (sum(xproc.quic_feed.frag_counts(n_payloads, P,
                                  "prefill" if prefill else "paced", reps)) // n_payloads),
                  engine_procs=E, dedup_depth=getattr(args, "dedup_depth", xproc.DEDUP_TCACHE_DEPTH))
    er, feed = r["engine"], r["feed"]
    n_total = r["txns"]
    wall = r["wall_s"]
    agg = er["stats"]
    res = {
        "metric": "verify mux tile end-to-end transactions/s, cross-process (quic process -> engine process -> "
                  "out links)",
        "tile": "fdgpu_vmux on fdt_mux_run in the engine process (python -m firedancer_amd.engine_proc); the GPU "
                "reads the payloads where the producer process wrote them (shared-memory links registered with the "
                "engines), parses, verifies and writes the out frags",
        "xproc": True, "pages": args.pages, "dedup_process": bool(args.dedup),
        "producers": P, "txns_per_s": round(n_total / wall, 1), "sigs_per_s": round(n_sig * n_total / n_payloads / wall, 1),
        "wall_s": round(wall, 4), "producer_s": round(max(feed["producer_s"]), 4),
        "producer_published": int(sum(feed["published"])), "gpus": args.gpus, "tiles": tiles_n,
        "batch_txn_max": batch, "inflight": inflight, "engines": tiles_n, "engine_slots": inflight,
        "engine_procs": E, "engine_pids": er["pid"],
        "batch_sig_max": getattr(args, "batch_sig_max", 0) or batch * 12, "rate_target": rate, "prefill": prefill,
        "link_depth": 1 << args.depth_lg, "offered_txns_per_s": None if prefill else feed["offered_per_s"],
        "stream_reps": reps, "lap_guard": int(args.lap_guard),
        "workload": "cfg3 (1-12 sigs/txn, payload <= 1232 B, 10% corrupted)" if getattr(args, "multi", 0)
        else "cfg1 (1 sig, msg U[180,220] B, 10% corrupted)",
        "txns": n_total, "sigs": n_sig * n_total // n_payloads, "batch_wait_us": args.wait_us,
        "cpus": cpus[:P + tiles_n + 1], "batch_latency_ms": er["batch_latency_ms"], "counters": agg,
        "mux": er["mux"], "expected_published": int((modes == 0).sum()) * (n_total // n_payloads),
        "in_huge_bytes": r["in_huge_bytes"], "engine_pid": er["pid"], "feed_pid": feed["pid"],
    }
    if "dedup" in r:
        # with the dedup in the loop the run is timed to its last frag (xproc: wall_s), and the verify -> dedup
        # links are reliable: every frag the verify tiles published must have reached it, nothing overrun
        res["dedup"] = r["dedup"]
        res["dedup_tcache_depth"] = getattr(args, "dedup_depth", xproc.DEDUP_TCACHE_DEPTH)
        ds = r["dedup"]["stats"]
        res["dedup_ok"] = (r["dedup"]["exit"] == 0 and ds["overrun"] == 0 and ds["corrupt"] == 0
                           and ds["in_frags"] == agg["published"] and ds["published"] + ds["dup"] == ds["in_frags"])
    res["published_ok"] = agg["published"] == res["expected_published"]
    return res


_NPZ = {"path": ""}


def start_producer(args, inl, arena, offs, sizes, rate, cpus, k=0):
    """The producer's C thread inherits the creating thread's CPU mask: pin
    this thread to cpus[k] around its start."""
    if not args.pin:
        return tile.Producer(inl, arena, offs, sizes, rate_tps=rate)
    keep = os.sched_getaffinity(0)
    os.sched_setaffinity(0, {cpus[k % len(cpus)]})
    try:
        return tile.Producer(inl, arena, offs, sizes, rate_tps=rate)
    finally:
        os.sched_setaffinity(0, keep)


def warm(engines, inflight, out_bytes=0, batch=64):
    """engine_proc.warm_engines: every ring slot warmed before the timed region"""
    from firedancer_amd.engine_proc import warm_engines
    warm_engines(engines, inflight, out_bytes=out_bytes, batch=batch)


def run_once(args, ps, arena, offs, sizes, n_sig, modes, tiles_n, batch, inflight, rate):
    if args.mux:
        return run_once_mux(args, ps, arena, offs, sizes, n_sig, modes, tiles_n, batch, inflight, rate)
    # one engine per tile thread, tiles spread over the GPUs
    engines = [fa.VerifyEngine(k % args.gpus, max_txn=batch, max_sig=batch * 12,
                               max_arena=batch * 1232, ring_depth=inflight) for k in range(tiles_n)]
    warm(engines, inflight)
    inl = tile.Link(1 << args.depth_lg, 1232)
    vts, vers = [], []
    for k in range(tiles_n):
        ver = tile.EngineVerifier([engines[k]])
        outl = tile.Link(1 << 12, tile.TPU_DCACHE_MTU)
        vts.append(tile.VerifyTile(inl, outl, ver, batch_txn_max=batch, inflight_max=inflight,
                                   batch_wait_us=args.wait_us, round_robin_idx=k, round_robin_cnt=tiles_n))
        vers.append((ver, outl))

    errs = []

    cpus = workload.physical_cpus()

    def run(vt, k):
        try:
            if args.pin:
                os.sched_setaffinity(0, {cpus[(1 + k) % len(cpus)]})   # this thread only
            vt.run(len(ps), timeout_s=300)
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    ths = [threading.Thread(target=run, args=(vt, k)) for k, vt in enumerate(vts)]
    start = time.perf_counter()
    prod = start_producer(args, inl, arena, offs, sizes, rate, cpus)
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    wall = time.perf_counter() - start
    n_pub, prod_s = prod.join()
    if errs:
        raise SystemExit(f"tile errors: {errs}")

    stats = [vt.stats() for vt in vts]
    lat = np.concatenate([vt.latencies_ns() for vt in vts]) / 1e6
    agg = {k: int(sum(s[k] for s in stats)) for k in stats[0]}
    res = {
        "metric": "verify tile end-to-end transactions/s (tango in -> GPU verify -> tango out)",
        "txns_per_s": round(len(ps) / wall, 1),
        "sigs_per_s": round(agg["sigs"] / wall, 1),
        "wall_s": round(wall, 4), "producer_s": round(prod_s, 4), "producer_published": int(n_pub),
        "gpus": args.gpus, "tiles": tiles_n, "batch_txn_max": batch, "inflight": inflight,
        "rate_target": rate, "workload": "cfg3 (1-12 sigs/txn, payload <= 1232 B, 10% corrupted)"
        if args.multi else "cfg1 (1 sig, msg U[180,220] B, 10% corrupted)",
        "txns": len(ps), "sigs": n_sig,
        "batch_latency_ms": {"p50": round(float(np.percentile(lat, 50)), 3),
                             "p99": round(float(np.percentile(lat, 99)), 3), "n": int(len(lat))},
        "counters": agg,
        "expected_published": int((modes == 0).sum()),
    }
    for vt in vts:
        vt.close()
    for ver, _ in vers:
        ver.close()
    for e in engines:
        e.close()
    return res


def run_once_mux(args, ps, arena, offs, sizes, n_sig, modes, tiles_n, batch, inflight, rate, cpus=None, device=None):
    """T verify mux tiles (fdt_mux_run threads) over one engine each, reading
    P quic->verify links (one producer thread each, the frags dealt round
    robin over the links, each paced at rate / P); the out links have no
    reliable consumer here (published frags count as consumed), so this
    measures ingest + verify + publish."""
    tpe = max(1, getattr(args, "tiles_per_engine", 1))
    # tiles sharing an engine share its `inflight` ring slots (each tile may hold up to all of them)
    engines = engine_pool(args, (tiles_n + tpe - 1) // tpe, batch, inflight, device)
    P = max(1, args.producers)
    lp = getattr(args, "link_pages", "") or None
    inls = [tile.Link(1 << args.depth_lg, 1232, pages=lp) for _ in range(P)]
    vms, vers = [], []
    for k in range(tiles_n):
        ver = tile.EngineVerifier([engines[k // tpe]])
        outl = tile.Link(1 << 14, tile.TPU_DCACHE_MTU, data_sz=tile.vmux_dcache_data_sz(1 << 14, batch, inflight),
                         pages=lp)
        guard = {} if getattr(args, "lap_guard", 1) else dict(lap_span_max=tile.LAP_OFF, lap_margin=tile.LAP_OFF)
        vms.append(tile.VerifyMuxTile(inls, outl, ver, batch_txn_max=batch, inflight_max=inflight,
                                      batch_wait_us=args.wait_us, round_robin_idx=k, round_robin_cnt=tiles_n,
                                      gpu_parse=int(args.gpu_parse), batch_sig_max=getattr(args, "batch_sig_max", 0),
                                      **guard))
        vers.append((ver, outl))
    cpus = cpus or workload.physical_cpus()[getattr(args, "cpu_offset", 0):] or workload.physical_cpus()
    # tile k's thread is pinned to cpus[P + k] (VerifyMuxTile.start inherits the caller's mask)
    # rate < 0: prefill -- every frag is published before the tiles start, so
    # the run measures the tiles' own drain rate (capacity), not the producers'
    prefill = rate < 0
    # a prefilled run gives every link the whole stream (link j starting a
    # j/P-th of the way in, so a txn's copies are far apart in every tile's
    # tcache window): P x N frags, long enough that the pipeline's fill and
    # drain do not dominate the drain time of several tiles
    reps = 1
    if prefill:
        # --prefill-reps R: each link's stream R times over (a small multi-signature set still gives a
        # run of ~100 batches; a txn's copies are a whole stream apart, far outside the tcache window,
        # so every copy is verified and published again)
        n = len(offs)
        reps = max(1, getattr(args, "prefill_reps", 1))
        feeds = [(np.tile(np.roll(offs, -(j * n // P)), reps), np.tile(np.roll(sizes, -(j * n // P)), reps))
                 for j in range(P)]
    else:
        # paced: link j carries every P-th frag, the stream published paced_reps times over (a txn's
        # copies are len(ps) frags apart: far outside the tiles' 16-deep tcache window)
        reps = max(1, getattr(args, "paced_reps", 1))
        feeds = [(np.tile(offs[j::P], reps), np.tile(sizes[j::P], reps)) for j in range(P)]
    n_total = sum(len(f[0]) for f in feeds)

    def start_tiles():
        for k, vm in enumerate(vms):
            vm.start(cpu=cpus[(P + k) % len(cpus)] if args.pin else None)

    # paced: the tiles are polling before the first frag is published (a producer that starts first
    # laps a tile still starting up: ~4 x the link depth lost in one run of r04k / r04n)
    if not prefill:
        start_tiles()
    start = time.perf_counter()
    prods = [start_producer(args, inls[j], arena, feeds[j][0], feeds[j][1], 0.0 if prefill else rate / P, cpus, j)
             for j in range(P)]
    if prefill:
        joined = [pr.join() for pr in prods]
        start = time.perf_counter()
        start_tiles()
    # done: every frag's outcome final -- or, when frags were lost to the
    # producers (lapped: the tiles log those too; skipped by the mux while it
    # lagged: never seen), the producers finished and the tiles sit idle with
    # no outcome added for 20 ms
    idle_since, last = None, -1
    while any(vm.final_cnt() < n_total for vm in vms):
        now = time.perf_counter()
        if now - start > 300:
            raise SystemExit("verify mux tiles timed out")
        cur = sum(vm.final_cnt() for vm in vms)
        if cur != last or not all(vm.idle() for vm in vms) or (not prefill and any(pr.running() for pr in prods)):
            idle_since, last = now, cur
        elif now - idle_since > 0.02:
            break
        time.sleep(0.0002)
    wall = (idle_since if idle_since is not None and any(vm.final_cnt() < n_total for vm in vms)
            else time.perf_counter()) - start
    for vm in vms:
        vm.stop()
    if not prefill:
        joined = [pr.join() for pr in prods]
    n_pub, prod_s = sum(j[0] for j in joined), max(j[1] for j in joined)
    stats = [vm.stats() for vm in vms]
    mstats = [vm.mux_stats() for vm in vms]
    lat = np.concatenate([vm.latencies_ns() for vm in vms]) / 1e6
    agg = {k: int(sum(s[k] for s in stats)) for k in stats[0]}
    agg["lap_margin_min"] = int(min(s["lap_margin_min"] for s in stats))
    agg["stall_max_ns"] = int(max(s["stall_max_ns"] for s in stats))
    # every frag lost to the producers: lapped before the device read it (the
    # tile's own count, FDGPU_CODE_LAPPED), skipped while the mux lagged, or
    # overwritten while the mux read its metadata
    agg["lapped"] = int(sum(s["lapped"] for s in stats))
    agg["overrun_polling"] = int(sum(m["overrun_polling"] for m in mstats))
    agg["overrun_reading"] = int(sum(m["overrun_reading"] for m in mstats))
    agg["overrun"] = agg["lapped"] + agg["overrun_polling"] + agg["overrun_reading"]
    res = {
        "metric": "verify mux tile end-to-end transactions/s (tango in -> GPU verify -> tango out)",
        "tile": "fdgpu_vmux on fdt_mux_run (mux callbacks; registered out dcache, no staging copy)"
                + {2: "; the GPU reads the payloads in the in dcache, parses, verifies and writes the out frags",
                   1: "; fd_txn_parse on the GPU", 0: "; fd_txn_parse on the tile core"}[int(args.gpu_parse)],
        "producers": P,
        "txns_per_s": round(n_total / wall, 1),
        "sigs_per_s": round(n_sig * n_total / len(ps) / wall, 1),
        "wall_s": round(wall, 4), "producer_s": round(prod_s, 4), "producer_published": int(n_pub),
        "gpus": args.gpus, "tiles": tiles_n, "batch_txn_max": batch, "inflight": inflight,
        "engines": len(engines), "engine_slots": inflight,
        "batch_sig_max": getattr(args, "batch_sig_max", 0) or batch * 12,
        "rate_target": rate, "prefill": prefill, "link_depth": 1 << args.depth_lg,
        # what the producers actually offered: frags published / their publishing time
        "offered_txns_per_s": round(n_pub / prod_s, 1) if prod_s > 0 and not prefill else None,
        "stream_reps": reps, "lap_guard": int(getattr(args, "lap_guard", 1)),
        "link_pages": lp or "numpy (first-touch)", "in_huge_bytes": [ln.huge_bytes() for ln in inls],
        "workload": "cfg3 (1-12 sigs/txn, payload <= 1232 B, 10% corrupted)" if getattr(args, "multi", 0) else "cfg1 (1 sig, msg U[180,220] B, 10% corrupted)",
        "txns": n_total, "sigs": n_sig * n_total // len(ps), "batch_wait_us": args.wait_us, "cpus": cpus[:P + tiles_n],
        "batch_latency_ms": {"p50": round(float(np.percentile(lat, 50)), 3) if len(lat) else None,
                             "p99": round(float(np.percentile(lat, 99)), 3) if len(lat) else None,
                             "n": int(len(lat))},
        "counters": agg, "mux": {k: int(sum(m[k] for m in mstats)) for k in mstats[0]},
        "expected_published": int((modes == 0).sum()) * (n_total // len(ps)),
    }
    res["published_ok"] = res["counters"]["published"] == res["expected_published"]
    for vm in vms:
        vm.close()
    for ver, _ in vers:
        ver.close()
    return res


_POOL = {}


def engine_pool(args, n, batch, inflight, device):
    """n engines (one per tile) for a run, kept across the runs of a sweep:
    a deployment opens its tiles' engines once, and a process that keeps
    opening and closing engines keeps creating HIP streams -- after a few
    dozen, new streams share hardware queues and batches of one tile
    serialise behind another's (a run after a 3-tile run took 2.5x as long
    per batch with the same kernel durations, profiles/r04/tile_run_order.md)."""
    key = (batch, inflight, device)     # (the flags are per process: a sweep's runs share them)
    pool = _POOL.setdefault(key, [])
    frag_bytes = (tile.TPU_DCACHE_MTU + 63) // 64 * 64
    new = []
    while len(pool) < n:
        k = len(pool)
        e = fa.VerifyEngine(device if device is not None else k % args.gpus, max_txn=batch, max_sig=batch * 12,
                            max_arena=batch * frag_bytes, ring_depth=inflight, pair=args.pair == 1,
                            pair_auto=args.pair == 2, merge=bool(getattr(args, "merge", 0)),
                            spread=getattr(args, "spread", 0) == 1, spread_auto=getattr(args, "spread", 0) == 2)
        if getattr(args, "reserve", 1):
            e.reserve()      # every slot sized for the largest batch now, not inside the run (as a tile's init does)
        pool.append(e)
        new.append(e)
    if new:
        warm(new, inflight, out_bytes=batch * frag_bytes if args.gpu_parse == 2 else 0, batch=batch)
    return pool[:n]


if __name__ == "__main__":
    sys.exit(main())
