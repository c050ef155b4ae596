"""Benchmark: verified Ed25519 signatures/s on MI355X (BASELINE.json metric).

Workload (BASELINE configs[1] = cfg2): 1M synthetic single-signature Solana
transactions per GPU (msg ~U[180,220] B, 90% valid / 10% with one bit flipped
in the signature, message or public key; seeded OpenSSL-signed, see
firedancer_amd/workload.py), staged in HBM before the timed region.  A step
is one full pass of the hot path over the batch: the signature kernel
(SHA-512, mod L, decode, small-order, [S]B - [k]A, compare) plus the per-txn
combine kernel, codes left in HBM.

Multi-GPU: one process per GPU (torch.distributed.run), each rank verifies its
own independent 1M batch (weak scaling, no data-path collective); CPU-side gloo
only for the barrier and the max-over-ranks time.

Extras on the JSON line: roofline (INT32 VALU, v_mad_u64_u32 issue peak),
cpu_baseline (the oracle, a C restatement, on this host's cores, N=1 only),
p50/p99 batch latency of 65,536-txn batches through the async PCIe path, and
the PCIe-inclusive pipelined throughput.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))

# HIP hardware queues, set before the runtime starts: every ring slot, device
# batch and tile engine owns a stream, and HIP maps a process's streams onto
# GPU_MAX_HW_QUEUES hardware queues (4 by default); two busy streams on one
# queue serialise.  This process (headline batches, latency ring slots) takes
# HW_QUEUES; the cfg5 tile lines run in a child process with TILE_HW_QUEUES
# for their two engines x eight slots (two tiles: 35 M txn/s with 16 queues,
# 44 M with 32, profiles/r03/mux_sweep/r03s_*.jsonl).  Every queue a process
# opens stays mapped on the device, so this process keeps to a few.
HW_QUEUES = 8
TILE_HW_QUEUES = 32
for _i, _a in enumerate(sys.argv):          # --hw-queues N (this process), read before HIP starts
    if _a.startswith("--hw-queues"):
        HW_QUEUES = int(_a.split("=", 1)[1] if "=" in _a else sys.argv[_i + 1])
os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES)
sys.path.insert(0, REPO)

# Algorithmic INT32 multiply-accumulates per signature:
# 3,300 field multiplications x 64 u32*u32 products (radix-2^32 schoolbook).
MADS_PER_SIG = 211_200
# v_mad_u64_u32 issue peak of one MI355X (the headline `peak`): 256 CU x 4
# SIMD x 16 lanes/clk (the instruction issues at half the 32-lane rate) x
# 2.4 GHz = 39.32 T/s.
VALU_MAD_PEAK_TOPS = 256 * 64 * 2.4e9 / 1e12
# The same instruction's measured throughput on MI355X (tools/ubench_int.hip,
# profiles/r01_ubench_int.jsonl: 55.15 lane-ops/CU/clk at 2.4 GHz, 8 waves
# per SIMD of independent chains) -- BASELINE.md's r_mad; `frac_measured`
# prices against it.
VALU_MAD_MEASURED_TOPS = 33.881


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--txns", type=int, default=1_000_000, help="transactions per GPU")
    ap.add_argument("--latency-batches", type=int, default=1000)   # >=1000 after 100 warm-up
    ap.add_argument("--latency-batch", type=int, default=65536)
    ap.add_argument("--cpu-sample", type=int, default=1_000_000, help="txns timed on the CPU oracle (bounded sample)")
    ap.add_argument("--no-extras", action="store_true", help="only the timed device-resident loop (profiling)")
    ap.add_argument("--hw-queues", type=int, default=HW_QUEUES,
                    help="GPU_MAX_HW_QUEUES of this process (applied before HIP starts; the tile child uses "
                         f"{TILE_HW_QUEUES})")
    ap.add_argument("--queues", type=int, default=2,
                    help="device batches verified round-robin, each on its own HIP stream (1: one stream)")
    ap.add_argument("--cfg3-txns", type=int, default=150_000,
                    help="multi-signature (cfg3) txns for the secondary device-resident line (0: skip)")
    ap.add_argument("--tile-cfg3-txns", type=int, default=250_000,
                    help="cfg3 txns for the tile lines' _cfg3 runs (0: skip them): ~1.6 M signatures, ~70 one-tile "
                         "batches, so the pipeline's fill and drain stay a small part of a run (150 K gave one tile "
                         "69 M sig/s against 86 M over 1 M txns; profiles/r05/tile_cfg3_cap.md)")
    ap.add_argument("--host-fed", type=int, default=1,
                    help="1: add the host-fed line (the cfg2 batch from host memory through the engine's ring)")
    ap.add_argument("--tile", type=int, default=1, help="1: add the cfg5 verify-tile lines (tango in -> GPU -> tango out)")
    ap.add_argument("--adv-txns", type=int, default=1_000_000,
                    help="txns of each adversarial batch (all equation failures / all corrupted R; 0: skip)")
    ap.add_argument("--keypool-txns", type=int, default=1_000_000,
                    help="txns of the signer-reuse batch (key pool of 4096) timed with and without the key "
                         "cache (0: skip)")
    ap.add_argument("--node-lines", type=int, default=0,
                    help="multi-rank runs: 1 adds the node-level cfg5 lines (bench.node_lines: one engine process "
                         "per GPU over shared links, the dedup over all of them); off by default, so a node's GPU "
                         "process count stays at the ranks' own")
    ap.add_argument("--node-procs", type=int, default=0,
                    help="engine processes of the node lines (0: one per rank; a one-GPU rehearsal keeps it small)")
    ap.add_argument("--ab-build", action="store_true",
                    help="let a library with A/B or fault-injection switches run (fdgpu_build_info; recorded in the "
                         "line as `build`); without it such a library is refused")
    return ap.parse_args()


class Dist:
    """Barrier + max-reduce across ranks (gloo over 127.0.0.1); no GPU collectives."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # gloo reports its connections on fd 1; keep stdout for the one JSON line
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x):
        if not self.dist:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x):
        if not self.dist:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()

    def cpus(self):
        """This rank's host cores: one logical CPU per physical core of its
        affinity, at most the box's 16-CPU share.  When ranks on the node
        see overlapping affinities (one process per GPU, unpinned), the union
        of physical cores is split into disjoint per-rank ranges, so the tile
        threads and the oracle of 8 ranks never share a core."""
        from firedancer_amd.workload import physical_cpus, idle_first, BOX_CPU_SHARE
        mine = physical_cpus(limit=1 << 20)
        if not self.dist:
            return idle_first(mine)[:BOX_CPU_SHARE]
        every = [None] * self.world
        self.dist.all_gather_object(every, mine)
        seen = set()
        overlap = False
        for c in every:
            overlap |= bool(seen & set(c))
            seen |= set(c)
        if not overlap:
            return idle_first(mine)[:BOX_CPU_SHARE]
        union = sorted(seen)
        k = max(1, len(union) // self.world)
        part = union[self.rank * k:(self.rank + 1) * k] or union[-k:]
        return part[:BOX_CPU_SHARE]


_T0 = time.monotonic()


def progress(msg, rank=0):
    """one progress line on stderr (stdout carries only the JSON line)"""
    print(f"[bench r{rank} {time.monotonic() - _T0:6.1f}s] {msg}", file=sys.stderr, flush=True)


def rank_seed(rank):
    """Each rank verifies its own independent cfg1 shard (weak scaling)."""
    from firedancer_amd import workload
    return workload.CFG1_SEED + rank


def aggregate(dist, n_sig, steps, dt):
    """Whole-job throughput: sigs of all ranks / the slowest rank's time."""
    dt_max = dist.max(dt)
    total = dist.sum(n_sig * steps)
    return total / dt_max, dt_max


FDGPU_ARENA_SLACK = 160   # readable bytes past a batch arena's last payload byte (fdgpu_internal.h)
RING_DEPTH = 8        # ring slots (one stream + workspace each) of the latency/PCIe engine (8: tools/pcie_probe.py)


def timed_batch(eng, a, t):
    """submit -> codes on the host, ms, and the part spent inside submit
    (descriptor expansion, staging copy, enqueue): the completion is watched
    with non-blocking polls (the completion word, as the verify tile polls),
    not a blocking event wait whose wake-up adds its own jitter"""
    t0 = time.perf_counter()
    tk = eng.submit(a, t)
    t1 = time.perf_counter()
    while eng.poll(tk, blocking=False) is None:
        pass
    return (time.perf_counter() - t0) * 1e3, (t1 - t0) * 1e3


def submit_parts(k):
    """p50/p99/max (ms) of the engine's per-call submit parts over its last k
    fdgpu_submit calls"""
    from firedancer_amd import _lib
    out = np.zeros(3 * k, dtype=np.uint64)
    n = int(_lib.lib().fdgpu_debug_submit_times(out.ctypes.data, k))
    t = out[:3 * n].reshape(n, 3) / 1e6
    return {name: [round(float(np.percentile(t[:, j], q)), 3) for q in (50, 99)] + [round(float(t[:, j].max()), 3)]
            for j, name in enumerate(("stage", "expand", "enqueue"))} if n else {}


def latency_and_pcie(eng, arena, txns, batch, nbatches, pin_cpu=None):
    """p50/p99 submit->codes-on-host latency of `batch`-txn batches (one in
    flight at a time), then pipelined throughput with every ring slot busy
    (PCIe-inclusive: host staging memcpy, uploads, kernels, code read-back).
    The latency loops run with Python's garbage collector off, so its pauses
    do not land in the tail."""
    import gc
    n = len(txns)
    starts = list(range(0, n - batch + 1, batch)) or [0]
    views = []
    for s in starts:
        t = txns[s:s + batch].copy()
        lo = int(t["sig_off"].min())
        hi = int((t["msg_off"] + t["msg_sz"]).max())
        for f in ("msg_off", "sig_off", "pub_off"):
            t[f] -= lo
        views.append((np.ascontiguousarray(arena[lo:hi]), t))
    for i in range(100):                                   # warm-up (starts the staging thread pool)
        a, t = views[i % len(views)]
        eng.verify_txns(a, t)
    # the submitting thread on one core for the timed loops (the staging
    # helpers, started above, keep the process's whole mask)
    keep = os.sched_getaffinity(0)
    if pin_cpu is not None:
        os.sched_setaffinity(0, {pin_cpu})
    gc.disable()
    lat = np.array([timed_batch(eng, *views[i % len(views)]) for i in range(nbatches)])
    gc.enable()
    parts = submit_parts(nbatches)
    def pipelined(vs):
        """every ring slot busy: submit -> poll over the batches, sigs/s"""
        sigs = 0
        t0 = time.perf_counter()
        inflight = []
        for i in range(max(len(vs), 4 * RING_DEPTH) * 2):
            a, t = vs[i % len(vs)]
            if len(inflight) == RING_DEPTH:
                eng.poll(inflight.pop(0), blocking=True)
            inflight.append(eng.submit(a, t))
            sigs += int(t["sig_cnt"].sum())
        for tk in inflight:
            eng.poll(tk, blocking=True)
        return sigs / (time.perf_counter() - t0)

    # host arena copied into the engine's pinned slots (fdgpu_submit's staging)
    pcie = pipelined(views)
    # the same batches in place in a host arena registered with the engine
    # (fdgpu_host_register): DMA'd straight from it, no staging copy
    eng.host_register(arena)
    reg_views = []
    for (_, t), s in zip(views, starts):
        lo = int(txns[s:s + batch]["sig_off"].min())
        reg_views.append((arena[lo:lo + int((t["msg_off"] + t["msg_sz"]).max())], t))
    pcie_reg = pipelined(reg_views)
    # the same latency measurement from the registered arena (DMA'd in place,
    # as the verify tile's registered out dcache is)
    gc.disable()
    lat_reg = np.array([timed_batch(eng, *reg_views[i % len(reg_views)]) for i in range(nbatches)])
    gc.enable()
    parts_reg = submit_parts(nbatches)
    eng.host_unregister(arena)
    os.sched_setaffinity(0, keep)

    def pct(x, q):
        return round(float(np.percentile(x, q)), 3)
    return {"p50_batch_latency_ms": pct(lat[:, 0], 50), "p99_batch_latency_ms": pct(lat[:, 0], 99),
            "p50_batch_latency_registered_ms": pct(lat_reg[:, 0], 50),
            "p99_batch_latency_registered_ms": pct(lat_reg[:, 0], 99),
            # where the tail sits: inside submit (host: expansion, staging) or after it (GPU, read-back, poll)
            "latency_split_ms": {"staged_submit_p50_p99": [pct(lat[:, 1], 50), pct(lat[:, 1], 99)],
                                 "staged_rest_p50_p99": [pct(lat[:, 0] - lat[:, 1], 50),
                                                         pct(lat[:, 0] - lat[:, 1], 99)],
                                 "registered_submit_p50_p99": [pct(lat_reg[:, 1], 50), pct(lat_reg[:, 1], 99)],
                                 "registered_rest_p50_p99": [pct(lat_reg[:, 0] - lat_reg[:, 1], 50),
                                                             pct(lat_reg[:, 0] - lat_reg[:, 1], 99)]},
            # inside submit, from the engine's own clock (fdgpu_debug_submit_times): staging copy,
            # descriptor expansion, enqueue of copies and launches -- p50 / p99 / max, ms
            "submit_parts_ms": {"staged": parts, "registered": parts_reg},
            "pcie_inclusive_sigs_per_s_per_gpu": round(pcie, 1),
            "pcie_inclusive_registered_sigs_per_s_per_gpu": round(pcie_reg, 1)}


HOST_FED_RING = 3       # 1M-txn slots of the host-fed engine: a batch's upload runs under the previous verify
HOST_FED_STEPS = 12


def host_fed(device, arena, txns, n_sig, ref_codes, value, steps=HOST_FED_STEPS, ring=HOST_FED_RING, pin_cpu=None):
    """The north-star shim path at the headline size (VERDICT r04 item 2;
    SURVEY 8(b)(ii), 8(d) "ingest is the only secondary bound"): the same
    cfg2 batch of 1M txns fed from HOST memory through the engine's ring
    (fdgpu_submit: per-signature expansion on the host, H2D upload, verify,
    codes back to the host), `ring` slots, each slot's upload overlapping the
    other slots' verifies; timed from the first submit to the last batch's
    codes on the host.  Two feeds: the arena registered with the engine
    (fdgpu_host_register: the upload is a DMA straight from it) and staged
    (copied into the slot's pinned arena by the engine's copy threads first).
    The H2D bytes per batch (arena + 16-B signature descriptors + 4-B
    permutation + 8-B txn descriptors) over the run give the achieved ingest
    rate, next to the link's own H2D rate measured in the same run."""
    from firedancer_amd import VerifyEngine, _lib
    L = _lib.lib()
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    n_txn = len(txns)
    eng = VerifyEngine(device, max_txn=n_txn, max_sig=n_sig, max_arena=arena.nbytes, ring_depth=ring)
    h2d_bytes = arena.nbytes + FDGPU_ARENA_SLACK + n_sig * (16 + 4) + n_txn * 8
    out = {"host_fed_batch_txns": n_txn, "host_fed_ring_slots": ring, "host_fed_steps": steps,
           "host_fed_h2d_bytes_per_batch": h2d_bytes}
    keep = os.sched_getaffinity(0)
    try:
        def feed(tag):
            ok = True
            tks = [eng.submit(arena, txns) for _ in range(ring)]            # every slot warm (workspace sized)
            for tk in tks:
                ok &= bool((eng.poll(tk, blocking=True) == ref_codes).all())
            if pin_cpu is not None:
                os.sched_setaffinity(0, {pin_cpu})
            tks, last = [], None
            t0 = time.perf_counter()
            for _ in range(steps):
                if len(tks) == ring:
                    last = eng.poll(tks.pop(0), blocking=True)
                tks.append(eng.submit(arena, txns))
            for tk in tks:
                last = eng.poll(tk, blocking=True)
            dt = time.perf_counter() - t0
            os.sched_setaffinity(0, keep)
            ok &= bool((last == ref_codes).all())
            parts = submit_parts(steps)
            out[f"host_fed_{tag}_sigs_per_s"] = round(steps * n_sig / dt, 1)
            out[f"host_fed_{tag}_ms_per_batch"] = round(dt / steps * 1e3, 3)
            out[f"host_fed_{tag}_h2d_gbps"] = round(steps * h2d_bytes / dt / 1e9, 2)
            out[f"host_fed_{tag}_submit_parts_ms"] = parts
            out[f"host_fed_{tag}_codes_equal"] = ok

        eng.host_register(arena)
        try:
            out["host_fed_h2d_link_gbps"] = round(L.fdgpu_debug_h2d_gbps(eng._h, arena.ctypes.data,
                                                                         min(arena.nbytes, 256 << 20), 10), 2)
            feed("registered")
        finally:
            eng.host_unregister(arena)
        feed("staged")
    finally:
        os.sched_setaffinity(0, keep)
        eng.close()
    out["host_fed_registered_vs_device_resident"] = round(out["host_fed_registered_sigs_per_s"] / value, 4)
    out["host_fed_staged_vs_device_resident"] = round(out["host_fed_staged_sigs_per_s"] / value, 4)
    out["host_fed_note"] = (f"{n_txn} cfg2 txns per batch from host memory through fdgpu_submit ({ring} ring slots: "
                            "expansion on the host, H2D, verify, codes back), first submit to last codes on the "
                            "host; registered: DMA straight from the registered arena; staged: copied into pinned "
                            "slots first; h2d_gbps: the batches' H2D bytes over the run; h2d_link_gbps: 256 MB "
                            "copies from the registered arena alone (HIP events)")
    return out


def latency_frag_io(eng, arena, txns, ref_codes, batch, nbatches, pin_cpu=None, views_n=4, keep_raw=False):
    """p50/p99 submit -> results-on-host latency of the verify tile's own
    path, gathered frag batches (fdgpu_submit_frags_io): `batch` raw payloads
    at 64-B chunk offsets of a registered "in dcache", read there by the
    device, parsed, verified, tagged and written back as out frags into a
    registered "out dcache" -- nothing staged or expanded on the host, so
    submit is validation + five launches.  One batch in flight, the
    submitting thread pinned, the garbage collector off; the library is
    called directly (no Python wrapper inside the timed region)."""
    import gc
    from firedancer_amd import _lib, tile, workload
    L = _lib.lib()
    n = min(len(txns), batch * views_n)
    ps = workload.payloads(arena, txns[:n])
    slots = [(len(p) + 63) // 64 * 64 for p in ps]
    in_off = np.concatenate([[0], np.cumsum(slots)])
    in_buf = tile._page_buf(int(in_off[-1]) + 4096)
    for p, o in zip(ps, in_off[:-1].tolist()):
        in_buf[o:o + len(p)] = np.frombuffer(p, dtype=np.uint8)
    caps = np.array([L.fdgpu_frag_out_cap(len(p)) for p in ps], dtype=np.uint64)
    views = []
    out_max = 0
    for b0 in range(0, n - batch + 1, batch):
        fio = np.zeros(batch, dtype=tile.FRAG_IO_DTYPE)
        fio["src"] = in_buf.ctypes.data + in_off[b0:b0 + batch]
        fio["sz"] = [len(p) for p in ps[b0:b0 + batch]]
        oo = np.concatenate([[0], np.cumsum((caps[b0:b0 + batch] + 63) // 64 * 64)])
        fio["out_off"], fio["out_cap"] = oo[:-1], caps[b0:b0 + batch]
        views.append((fio, int(oo[-1]), b0))
        out_max = max(out_max, int(oo[-1]))
    out_buf = tile._page_buf(out_max + 4096)
    codes = np.zeros(batch, dtype=np.int8)
    tags = np.zeros(batch, dtype=np.uint64)
    osz = np.zeros(batch, dtype=np.uint16)
    cp, tp, op, ob = codes.ctypes.data, tags.ctypes.data, osz.ctypes.data, out_buf.ctypes.data
    eng.host_register(in_buf)
    eng.host_register(out_buf)
    keep = os.sched_getaffinity(0)
    try:
        def one(v):
            fio, osz_b, _ = v
            t0 = time.perf_counter()
            tk = L.fdgpu_submit_frags_io(eng._h, fio.ctypes.data, batch, ob, osz_b, 0x5EED, None, 0)
            t1 = time.perf_counter()
            if tk < 0:
                raise RuntimeError(f"fdgpu_submit_frags_io: {tk} ({_lib.last_error()})")
            while True:
                rc = L.fdgpu_poll_frags_io(eng._h, tk, cp, tp, op, 0)
                if rc != 1:
                    break
            if rc:
                raise RuntimeError(f"fdgpu_poll_frags_io: {rc}")
            return (time.perf_counter() - t0) * 1e3, (t1 - t0) * 1e3
        for i in range(50):                                # warm every slot (buffers sized on first use)
            one(views[i % len(views)])
        ok = True
        for v in views:                                    # the codes, against the device-resident batch's
            one(v)
            ref = ref_codes[v[2]:v[2] + batch]
            parsed = codes != tile.CODE_PARSE_FAIL
            ok &= bool((codes[parsed] == ref[parsed]).all()) and int((~parsed).sum()) < batch // 100
        if pin_cpu is not None:
            os.sched_setaffinity(0, {pin_cpu})
        gc.disable()
        lat = np.array([one(views[i % len(views)]) for i in range(nbatches)])
        gc.enable()
    finally:
        os.sched_setaffinity(0, keep)
        eng.host_unregister(in_buf)
        eng.host_unregister(out_buf)

    def pct(x, q):
        return round(float(np.percentile(x, q)), 3)
    out = {"p50_batch_latency_gathered_ms": pct(lat[:, 0], 50), "p99_batch_latency_gathered_ms": pct(lat[:, 0], 99),
           "latency_split_gathered_ms": {"submit_p50_p99": [pct(lat[:, 1], 50), pct(lat[:, 1], 99)],
                                         "rest_p50_p99": [pct(lat[:, 0] - lat[:, 1], 50),
                                                          pct(lat[:, 0] - lat[:, 1], 99)]},
           "gathered_codes_equal": ok}
    if keep_raw:
        out["lat_ms"] = [round(float(x), 4) for x in lat[:, 0]]
    return out


def sync_latency(arena, txns, calls=1000, threads=64):
    """The synchronous drop-in API (fd_ed25519_verify through the C ABI,
    fd_ed25519.h:96-101): p50/p99 of `calls` sequential calls on one thread
    (one GPU round trip each), then `threads` threads calling concurrently
    (the engine coalesces concurrent calls into one batch per round trip)."""
    import threading
    from firedancer_amd import _lib, ed25519
    L = _lib.lib()
    recs = []
    for t in txns[:max(calls, threads * 16)]:
        m = arena[int(t["msg_off"]):int(t["msg_off"]) + int(t["msg_sz"])].tobytes()
        recs.append((m, arena[int(t["sig_off"]):int(t["sig_off"]) + 64].tobytes(),
                     arena[int(t["pub_off"]):int(t["pub_off"]) + 32].tobytes()))
    for m, sg, pb in recs[:50]:                                        # warm-up (engine open)
        L.fd_ed25519_verify(m, len(m), sg, pb, None)
    lat = []
    for m, sg, pb in recs[:calls]:
        t0 = time.perf_counter()
        L.fd_ed25519_verify(m, len(m), sg, pb, None)
        lat.append((time.perf_counter() - t0) * 1e6)
    per = len(recs) // threads
    before = ed25519.sync_stats()

    def worker(k):
        for m, sg, pb in recs[k * per:(k + 1) * per]:
            L.fd_ed25519_verify(m, len(m), sg, pb, None)
    ths = [threading.Thread(target=worker, args=(k,)) for k in range(threads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    after = ed25519.sync_stats()
    lat = np.array(lat)
    n_conc = after["calls"] - before["calls"]
    return {"sync_call_latency_us_p50": round(float(np.percentile(lat, 50)), 1),
            "sync_call_latency_us_p99": round(float(np.percentile(lat, 99)), 1),
            "sync_calls": calls,
            "sync_concurrent_threads": threads,
            "sync_concurrent_calls_per_s": round(n_conc / dt, 1),
            "sync_concurrent_calls_per_batch": round(n_conc / max(1, after["batches"] - before["batches"]), 2),
            "sync_errors": after["errors"],
            "sync_note": "fd_ed25519_verify via ctypes, cfg1 single-signature txns; sequential: one GPU round "
                         "trip per call; concurrent: calls coalesced into shared batches (group commit)"}


TILE_RUNS = (  # name, verify tiles, quic links (producers), offered txn/s (-1: prefilled links, the tiles' capacity)
    # the paced runs first, so a latency line never runs behind a capacity run's multi-GB prefill; at most
    # two engines (18 streams) in the child: three at 32 HW queues slowed every later run in the process
    # (profiles/r04/tile_run_order.md)
    ("mux1_paced_12M", 1, 2, 12e6),
    ("mux1_paced_16M", 1, 2, 16e6),
    ("mux2_paced_20M", 2, 4, 20e6),
    ("mux2_paced_24M", 2, 4, 24e6),
    # the reference's link depth near the producers' limit (~9-12 M frags/s a thread): what two tiles sustain
    # with nothing lost at 16384 deep
    ("mux2_paced_36M", 2, 4, 36e6),
    ("mux1_capacity", 1, 1, -1.0),
    ("mux2_capacity", 2, 2, -1.0),
)
# quic -> verify link depth: paced runs at the reference's (config->tiles.verify.receive_buffer_size,
# default.toml:888-893: 16384, fd_frankendancer.c:59), with the stream published TILE_PACED_REPS times
# over (>= 30 x the depth per link: the producers can lap the tiles); capacity runs prefill every frag
# before the tiles start, so their links hold the whole stream
TILE_DEPTH_LG_PACED, TILE_DEPTH_LG_PREFILL, TILE_PACED_REPS = 14, 21, 4
TILE_BATCH, TILE_INFLIGHT = 16384, 8   # txns per GPU batch, batches in flight per tile
# tile engines: FDGPU_FLAG_PAIR_AUTO -- the two-lane verify while an engine's batches leave the GPU idle
# (paced: p50 batch latency 1.13 vs 1.40 ms at 12 M txn/s, 1.47 vs 1.81 at 24 M; capacity unchanged;
# profiles/r04/tile_pair.md)
TILE_PAIR = 2
# ... and FDGPU_FLAG_SPREAD_AUTO: one verify block per CU while an engine's batches fit the chip that way
# (concurrent small launches otherwise stack two blocks per CU; profiles/r04/spread.md)
TILE_SPREAD = 2
# multi-signature frags: a batch also closes at this many signatures by the frag-size bound the tile sees
# (~9.5 per cfg3 frag for ~6.5 real).  With the gathered kernels on 16 workgroups (round 5) one tile
# reaches 86 M sig/s at 32768 (p99 3.0 ms) against 70.5 M at 24576, and two tiles 91 M at 24576 each
# (p99 5.1 ms; 32768: 90 M at p99 8.6-12 ms, 49152: 90 M at 10 ms; profiles/r05/tile_cfg3_cap.md)
TILE_CFG3_SIG_MAX = 32768
TILE_CFG3_SIG_MAX_BY_TILES = {1: 32768, 2: 24576}
# the cfg3 capacity runs publish their 250 K-txn stream this many times over into each link (every
# copy verified and published again: they are a stream apart, outside the tiles' 16-deep tcache),
# ~100+ batches a run, so the pipeline's fill and drain do not weigh (150-250 K txns once: one tile
# 69-74 M sig/s against 86 M over 1 M distinct txns; profiles/r05/tile_cfg3_cap.md)
TILE_CFG3_PREFILL_REPS = 4
TILE_RUNS_CFG3 = (  # the same tile over cfg3 frags (1-12 signatures, payloads up to the 1232-B MTU: SURVEY 8(d) cfg5)
    ("mux1_capacity_cfg3", 1, 1, -1.0),
    ("mux2_capacity_cfg3", 2, 2, -1.0),
)


TILE_REPS = 5   # a capacity run drains 1M frags in a few tens of ms: the median of five
# the deployable shape: the same tile as the engine process
# (python -m firedancer_amd.engine_proc) over shared-memory links that a producer
# process (tools/quic_feed.py) publishes into, every page faulted in before the
# run; each run starts both processes (engine open + warm-up ~3 s), so three runs each
# Fields after the rate: engine processes sharing the links (tiles / E each, global round-robin shares --
# the multi-GPU form of the stage, here on this rank's one GPU) and 1 when the sandboxed dedup process reads
# every verify -> dedup link reliably at the reference's tcache depth (4,194,302, default.toml:910): the
# e2e lines are timed to the dedup's last frag (fd_frankendancer.c:136, the node's verify -> dedup path)
TILE_RUNS_XPROC = (
    ("xproc_mux1_paced_16M", 1, 2, 16e6),
    ("xproc_mux2_paced_24M", 2, 4, 24e6),
    ("xproc_mux1_capacity", 1, 1, -1.0),
    ("xproc_mux2_capacity", 2, 2, -1.0),
    ("xproc_2proc_capacity", 2, 2, -1.0, 2, 0),
    ("xproc_2proc_paced_12M", 2, 4, 12e6, 2, 0),
    ("xproc_e2e_dedup_capacity", 2, 2, -1.0, 1, 1),
    ("xproc_e2e_dedup_paced_2M", 2, 4, 2e6, 1, 1),
)
TILE_REPS_XPROC = 3
TILE_DEPTH_LG_PREFILL_XPROC = 21      # as the in-process capacity lines: the lap guard never sees a prefilled frag at risk


def tile_cmd(rank, cpus, npz, out, runs=TILE_RUNS, multi=0, xproc=False):
    """tools/bench_tile.py's command line for the cfg5 runs (tests/test_bench_cli.py
    parses it with bench_tile's own parser).  The tiles run in a child process:
    its HIP runtime gives the tile engines' slot streams hardware queues of
    their own, instead of the ones this process's headline, latency and ingest
    engines already hold (shared queues serialise the tiles' batches).  The
    child picks its GPU as rank % the devices it sees (--device-rank): this
    process has not started a HIP runtime when the child runs, so a node of
    N ranks has at most N GPU processes at any time (a rank's own engines
    open only after its child has exited)."""
    sweep = ";".join(f"{tiles_n},{TILE_BATCH},{TILE_INFLIGHT},{rate:g},{prods}" +
                     (f",{TILE_CFG3_SIG_MAX_BY_TILES.get(tiles_n, TILE_CFG3_SIG_MAX)}" if multi else
                      f",0,{rest[0]},{rest[1]}" if rest else "")
                     for _, tiles_n, prods, rate, *rest in runs)
    cmd = [sys.executable, os.path.join(REPO, "tools", "bench_tile.py"), "--mux", "1", "--gpu-parse", "2",
           "--multi", str(int(multi)), "--producers-same-as-tiles", "1", "--depth-lg", str(TILE_DEPTH_LG_PREFILL),
           "--depth-lg-paced", str(TILE_DEPTH_LG_PACED), "--paced-reps", str(TILE_PACED_REPS),
           "--wait-us", "200", "--pin", "1", "--hw-queues", str(TILE_HW_QUEUES), "--warm-runs", "0" if xproc else "1",
           "--reps", str(TILE_REPS_XPROC if xproc else TILE_REPS),
           "--pair", str(TILE_PAIR), "--spread", str(TILE_SPREAD),
           "--payload-npz", npz, "--device-rank", str(rank), "--sweep", sweep, "--out", out]
    if multi:
        cmd += ["--batch-sig-max", str(TILE_CFG3_SIG_MAX), "--prefill-reps", str(TILE_CFG3_PREFILL_REPS)]
    if xproc:
        cmd += ["--xproc", "1", "--pages", "4k", "--depth-lg", str(TILE_DEPTH_LG_PREFILL_XPROC)]
    if cpus:
        cmd += ["--cpu-list", ",".join(str(c) for c in cpus)]
    return cmd


def _tile_child(rank, cpus, arena, txns, modes, runs, tag=""):
    xp = tag == "xproc"
    runs = tuple(runs)
    reps_n = TILE_REPS_XPROC if xp else TILE_REPS
    """tools/bench_tile.py in a child process over these txns as raw frags:
    {tile_<name>_...} per run (median of TILE_REPS)."""
    import subprocess
    import tempfile
    from firedancer_amd import workload
    ps = workload.payloads(arena, txns)
    parena, poffs, psizes = workload.pack_payloads(ps)
    out = {}
    with tempfile.TemporaryDirectory() as td:
        npz, res_path = os.path.join(td, "frags.npz"), os.path.join(td, "tile.jsonl")
        np.savez(npz, arena=parena, offs=poffs, sizes=psizes, modes=modes, n_sig=int(txns["sig_cnt"].sum()))
        # the child's per-run lines are echoed to stderr as they come (a long bench stays visibly alive)
        err_path = os.path.join(td, "tile.err")
        with open(err_path, "w") as err:
            p = subprocess.Popen(tile_cmd(rank, cpus, npz, res_path, runs, multi=tag == "cfg3", xproc=xp),
                                 stdout=subprocess.PIPE, stderr=err, text=True)
            import threading
            killer = threading.Timer(600, p.kill)          # the child's time limit
            killer.start()
            for ln in p.stdout:
                if ln.startswith("{"):
                    try:
                        x = json.loads(ln)
                        ln = f"tiles {x.get('tiles')} producers {x.get('producers')}: {x.get('txns_per_s')} txn/s"
                    except ValueError:
                        pass
                progress(f"tile{('_' + tag) if tag else ''} {ln.strip()[:160]}", rank)
            rc = p.wait()
            killer.cancel()
        if rc not in (0, 1) or not os.path.exists(res_path):
            raise RuntimeError(f"tools/bench_tile.py failed ({rc}): {open(err_path).read()[-2000:]}")
        res_all = [json.loads(x) for x in open(res_path) if x.strip()]
    if len(res_all) != len(runs) * reps_n:
        raise RuntimeError(f"tools/bench_tile.py gave {len(res_all)} runs, expected {len(runs) * reps_n}")
    for i, (name, tiles_n, prods, rate, *rest) in enumerate(runs):
        reps = res_all[i * reps_n:(i + 1) * reps_n]
        assert all(x["tiles"] == tiles_n and x["producers"] == prods for x in reps)
        if rest:
            assert all(x["engine_procs"] == rest[0] and ("dedup" in x) == bool(rest[1]) for x in reps)
            out[f"tile_{name}_engine_procs"] = rest[0]
        res = sorted(reps, key=lambda x: x["txns_per_s"])[len(reps) // 2]
        out[f"tile_{name}_txns_per_s_runs"] = [x["txns_per_s"] for x in reps]
        lat = res["batch_latency_ms"]
        out[f"tile_{name}_txns_per_s"] = res["txns_per_s"]
        if tag == "cfg3":
            out[f"tile_{name}_sigs_per_s"] = res["sigs_per_s"]
            out[f"tile_{name}_batch_sig_max"] = res["batch_sig_max"]
        out[f"tile_{name}_batch_latency_ms_p50_p99"] = [lat["p50"], lat["p99"]]
        out[f"tile_{name}_link_depth"] = res["link_depth"]
        if rate > 0:       # what the producers achieved (the line's name is the rate asked of them)
            out[f"tile_{name}_offered_txns_per_s"] = res["offered_txns_per_s"]
        # frags lost to the producers, worst of the runs: overruns = lapped (before the device read
        # them) + skipped while the mux lagged + overwritten while it read their metadata
        out[f"tile_{name}_overruns"] = max(x["counters"]["overrun"] for x in reps)
        out[f"tile_{name}_lapped"] = max(x["counters"]["lapped"] for x in reps)
        out[f"tile_{name}_rescued"] = max(x["counters"]["rescued"] for x in reps)
        out[f"tile_{name}_parse_fail"] = res["counters"]["parse_fail"]
        out[f"tile_{name}_published_ok"] = all(x["published_ok"] for x in reps)
        if rest and rest[1]:           # the dedup tile in the loop, reliable links, the reference's depth
            out[f"tile_{name}_dedup_ok"] = all(x["dedup_ok"] for x in reps)
            out[f"tile_{name}_dedup_tcache_depth"] = res["dedup_tcache_depth"]
            ds = res["dedup"]["stats"]
            out[f"tile_{name}_dedup_in_published_dup"] = [ds["in_frags"], ds["published"], ds["dup"]]
        # the tile's longest gap between two of its polls, worst of the runs: a core taken away (another
        # tenant's thread on it, the runtime blocking) -- a paced link laps a tile stalled for
        # depth / per-link rate (16384 / 5 M/s = 3.3 ms)
        out[f"tile_{name}_stall_max_ms"] = round(max(x["counters"].get("stall_max_ns", 0) for x in reps) / 1e6, 2)
        if rate > 0:
            # the fewest publishes any batch's oldest frag had left before its line's reuse, seen when the
            # batch completed (after the device read it), in ms at the link's offered rate; worst of the runs
            lm = min(x["counters"]["lap_margin_min"] for x in reps)
            out[f"tile_{name}_lap_margin_min_seqs"] = lm if lm < 2 ** 63 else None
            out[f"tile_{name}_lap_margin_min_seqs_runs"] = [x["counters"]["lap_margin_min"] if
                                                            x["counters"]["lap_margin_min"] < 2 ** 63 else None
                                                            for x in reps]
            per_link = min(x["offered_txns_per_s"] / x["producers"] for x in reps if x.get("offered_txns_per_s"))
            out[f"tile_{name}_lap_margin_min_ms"] = round(lm / per_link * 1e3, 3) if lm < 2 ** 63 else None
    return out


def xproc_runs(world):
    """The cross-process lines a rank runs: with several ranks on a node, not
    the ones that start two engine processes (8 ranks x 2 would be 16 GPU
    processes at once; a rank's own engines open only after its tile lines,
    so one engine process per rank keeps the node at one per GPU)."""
    return TILE_RUNS_XPROC if world == 1 else tuple(r for r in TILE_RUNS_XPROC if not (len(r) > 4 and r[4] > 1))


NODE_RUNS = (  # name, quic links (producers), offered txn/s (-1: prefilled), runs -- one tile per GPU of the node
    ("node_e2e_dedup_capacity", 2, -1.0, 2),
    ("node_e2e_dedup_paced_2M", 4, 2e6, 2),
)


def node_lines(dist, arena, txns, modes, cpus, engine_cmd=None, depth_lg=None, batch=TILE_BATCH,
               inflight=TILE_INFLIGHT, procs=None):
    """BASELINE cfg5 at the node's scale (world > 1; rank 0 runs it while the
    other ranks wait at a barrier, before any rank starts a HIP runtime of its
    own): verify_tile_cnt = world -- one engine process per GPU, one tile each
    as global tile r of world over the same quic -> verify links
    (fd_frankendancer.c:99,131-133, fd_verify.c:46), each inside its seccomp
    policy -- and the one sandboxed dedup tile over every verify -> dedup link,
    reliably, at the reference's tcache depth; timed from the first frag to the
    dedup's last.  Every frag's outcome reaches the dedup or the run is not ok.
    engine_cmd / depth_lg (prefill, paced) / batch / inflight: the CPU test's
    stand-in engine and small links (tests/_multirank_worker.py).  procs:
    engine processes (default one per rank; engine process k on device
    rank k)."""
    depth_lg = depth_lg or (TILE_DEPTH_LG_PREFILL, TILE_DEPTH_LG_PACED)
    procs = procs or dist.world
    import tempfile
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import xproc
    from firedancer_amd import workload
    every = [None] * dist.world
    dist.dist.all_gather_object(every, list(cpus or []))
    node_cpus = sorted(set(c for cs in every for c in cs))
    out = {}
    if dist.rank == 0:
        ps = workload.payloads(arena, txns)
        pa, po, psz = workload.pack_payloads(ps)
        with tempfile.TemporaryDirectory() as td:
            npz = os.path.join(td, "frags.npz")
            np.savez(npz, arena=pa, offs=po, sizes=psz)
            exp_once = int((modes == 0).sum())
            for name, P, rate, reps_n in NODE_RUNS:
                prefill = rate < 0
                reps = 1 if prefill else TILE_PACED_REPS
                depth = 1 << (depth_lg[0] if prefill else depth_lg[1])
                mult = sum(xproc.quic_feed.frag_counts(len(ps), P, "prefill" if prefill else "paced", reps)) // len(ps)
                runs = []
                for _ in range(reps_n):
                    r = xproc.run(npz, len(ps), tiles=procs, producers=P, mode="prefill" if prefill else "paced",
                                  rate=0.0 if prefill else rate, reps=reps, depth=depth, batch=batch,
                                  inflight=inflight, pair=TILE_PAIR, spread=TILE_SPREAD, dedup=True,
                                  engine_cmd=engine_cmd,
                                  dedup_frags=exp_once * mult, engine_procs=procs,
                                  proc_device_ranks=list(range(procs)),
                                  cpus=node_cpus[:P + procs + 1] if len(node_cpus) > P + procs else None,
                                  timeout=300)
                    st, ds = r["engine"]["stats"], r["dedup"]["stats"]
                    runs.append({"txns_per_s": r["txns_per_s"], "published": st["published"],
                                 "published_ok": st["published"] == exp_once * mult,
                                 "dedup_ok": (r["dedup"]["exit"] == 0 and ds["overrun"] == 0 and
                                              ds["in_frags"] == st["published"] and
                                              ds["published"] + ds["dup"] == ds["in_frags"]),
                                 "overrun": st["overrun"], "dedup": [ds["in_frags"], ds["published"], ds["dup"]],
                                 "lat": r["engine"]["batch_latency_ms"]})
                med = sorted(runs, key=lambda x: x["txns_per_s"])[len(runs) // 2]
                out[f"tile_{name}_txns_per_s"] = med["txns_per_s"]
                out[f"tile_{name}_txns_per_s_runs"] = [x["txns_per_s"] for x in runs]
                out[f"tile_{name}_published_ok"] = all(x["published_ok"] for x in runs)
                out[f"tile_{name}_dedup_ok"] = all(x["dedup_ok"] for x in runs)
                out[f"tile_{name}_overruns"] = max(x["overrun"] for x in runs)
                out[f"tile_{name}_dedup_in_published_dup"] = med["dedup"]
                out[f"tile_{name}_batch_latency_ms_p50_p99_worst_gpu"] = [med["lat"]["p50"], med["lat"]["p99"]]
        out["tile_node_config"] = (f"{procs} engine processes, one per GPU (--device-rank r), one verify tile each "
                                   f"as global tile r of {procs} over the same quic -> verify links (P per line), "
                                   "each in its seccomp policy; the sandboxed dedup over every verify -> dedup link at "
                                   "tcache depth 4194302; capacity: links prefilled 2^21 deep; paced: 16384-deep links, "
                                   f"the stream {TILE_PACED_REPS}x over; cfg1 frags of rank 0; median of the runs")
    dist.barrier()
    return out


def tile_lines(rank, arena, txns, modes, cpus, cfg3=None, world=1):
    """BASELINE configs[4] (cfg5) on this rank's GPU: the verify tile in the
    reference's shape -- the fd_verify.c:232-246 callbacks (fdgpu_vmux) on
    the mux loop (fdt_mux_run, FD_MUX_FLAG_COPY | MANUAL_PUBLISH), tcache and
    publish in order -- with the byte work on the GPU (gpu_parse 2,
    fdgpu_submit_frags_io): the device reads each payload in the registered
    in dcache, parses, verifies, tags it and writes the out frag into the
    registered out dcache; the tile core only moves frag metadata.  Over
    this rank's cfg1 txns as raw frags (TILE_RUNS) and, given `cfg3`, over
    the cfg3 txns too (TILE_RUNS_CFG3, SURVEY 8(d)'s cfg5 generator).  T
    tiles read P quic->verify links round robin (P = T for capacity, 2T
    paced: one producer thread copies ~12 M frags/s; every verify tile reads
    every QUIC tile's link, fd_frankendancer.c:131-133), one engine per tile
    on this GPU, 16K-txn batches, 8 in flight, producers and tiles pinned to
    their own cores, in a child process (tile_cmd).  Every run checks that
    exactly the verified txns were published."""
    from firedancer_amd.workload import same_l3_first
    # producers and tiles of a run on one CCD when one has room (a tile and its producers on two
    # sockets ran a quarter slower, profiles/r04/tile_host_cost.md)
    cpus = same_l3_first(list(cpus), 6) if cpus else cpus
    out = _tile_child(rank, cpus, arena, txns, modes, TILE_RUNS)
    out["tile_mux2_vs_mux1_capacity"] = round(out["tile_mux2_capacity_txns_per_s"] /
                                              out["tile_mux1_capacity_txns_per_s"], 3)
    if cfg3 is not None:
        out.update(_tile_child(rank, cpus, *cfg3, TILE_RUNS_CFG3, tag="cfg3"))
        out["tile_cfg3_txns"] = len(cfg3[1])
    # the deployable shape: producers and tiles in separate processes
    out.update(_tile_child(rank, cpus, arena, txns, modes, xproc_runs(world), tag="xproc"))
    for name, inproc in (("xproc_mux1_paced_16M", "mux1_paced_16M"), ("xproc_mux2_paced_24M", "mux2_paced_24M")):
        out[f"tile_{name}_vs_in_process"] = round(out[f"tile_{name}_txns_per_s"] / out[f"tile_{inproc}_txns_per_s"], 3)
    out["tile_xproc_config"] = ("the same tile in the engine process (python -m firedancer_amd.engine_proc) over "
                                "/dev/shm links a separate producer process (tools/quic_feed.py) publishes into, "
                                "every link page faulted in before the run (4 KB pages: this host offers no shared "
                                "2 MB pages, tile.hugepage_support()); paced: the reference's 16384-deep links; "
                                f"capacity: one 2^{TILE_DEPTH_LG_PREFILL_XPROC}-deep link per tile prefilled by the "
                                "producer process; the engine process inside its seccomp policy once its tiles run "
                                "(engine_proc --sandbox 1); _2proc_: two engine processes, one tile each, as global "
                                "tiles 0 and 1 of 2 over the same links (--rr-idx/--rr-cnt: the multi-GPU form, here "
                                "on this rank's GPU; single-rank runs only); _e2e_dedup_: the sandboxed dedup process "
                                "reads both out links reliably at the reference's tcache depth (4194302) and the run "
                                "is timed to its last frag (_dedup_in_published_dup: frags in, published, dropped as "
                                f"duplicates); median of {TILE_REPS_XPROC} runs, each starting every process")
    out["tile_config"] = ("fdgpu_vmux on fdt_mux_run (the reference's mux-callback verify tile), payload gather, "
                          "fd_txn_parse, verify, dedup tag and out-frag assembly on the GPU; muxT: T verify tiles "
                          "reading P quic->verify links (one producer thread each; P = T for capacity, 2T paced), one engine "
                          "per tile on this GPU, "
                          f"cfg1 frags (_cfg3: cfg3 frags, batches closed at _batch_sig_max signatures by the frag-size "
                          f"bound: half-size for two tiles), {TILE_BATCH}-txn batches, {TILE_INFLIGHT} in flight, {TILE_HW_QUEUES} HIP hardware "
                          "queues, in a child process (tools/bench_tile.py); capacity: every frag published into "
                          f"2^{TILE_DEPTH_LG_PREFILL}-deep links before the tiles start, timed from tile start to the "
                          f"last outcome; paced_R: R txn/s asked of the producers in total (achieved: _offered_txns_per_s) "
                          f"into {1 << TILE_DEPTH_LG_PACED}-deep links (the reference's receive_buffer_size) while the "
                          f"tiles run, the stream published {TILE_PACED_REPS}x over; the lap guard on; overruns count "
                          f"every frag lost to the producers (_lapped: before the GPU read it); median of {TILE_REPS} "
                          "runs each")
    return out


def gpu_ingest(eng, arena, txns, ref_codes):
    """SURVEY 8(f) row 3 on the device: the same cfg2 txns as raw payloads
    ([sig_cnt][sigs][message], as the quic tile hands them over), parsed,
    scanned and expanded on the GPU (fdgpu_dev_batch_upload_frags) before the
    verify; HIP-event times of the ingest kernels and the verify, and the
    codes against the descriptor path's (already checked against the oracle)."""
    from firedancer_amd.ed25519 import FRAG_DTYPE
    frags = np.zeros(len(txns), dtype=FRAG_DTYPE)
    frags["off"] = txns["sig_off"] - 1
    frags["sz"] = txns["msg_off"] + txns["msg_sz"] - frags["off"]
    from firedancer_amd import tile
    from firedancer_amd.ed25519 import CODE_PARSE_FAIL
    fb = eng.upload_frags(arena, frags)
    fb.verify()
    got = fb.codes()
    _, ing, ver, comb = fb.time2(5)
    n_sig = fb.n_sig
    _, tsz = fb.txns(records=False)
    fb.free()
    # algorithmic HBM bytes of the ingest kernels: payloads read, fd_txn_t
    # records written, per-txn records (frag 8 + txn record 20 + count 4 +
    # first-signature 4 (x2: scan and expand) + combine item 8 + footprint 2)
    # and 16-B signature descriptors written
    ing_bytes = int(frags["sz"].sum()) + int(tsz.sum()) + len(frags) * 50 + n_sig * 16
    # a corrupted message byte can leave a payload that is not a transaction:
    # the verify tile drops it at parse (FDGPU_CODE_PARSE_FAIL here) where the
    # descriptor path verifies it; every such frag must fail the host parser
    # too, and every other code must equal the descriptor path's
    pf = np.flatnonzero(got == CODE_PARSE_FAIL)
    offs, sizes = frags["off"].astype(np.int64), frags["sz"].astype(np.int64)
    host_pf_ok = all(tile.txn_parse(arena[offs[i]:offs[i] + sizes[i]].tobytes())[0] == 0 for i in pf)
    rnd = np.random.default_rng(7).choice(len(txns), size=min(2000, len(txns)), replace=False)
    host_ok = all(tile.txn_parse(arena[offs[i]:offs[i] + sizes[i]].tobytes())[0] != 0 for i in rnd if got[i] != CODE_PARSE_FAIL)
    mism = int(((got != ref_codes) & (got != CODE_PARSE_FAIL)).sum()) + (0 if host_pf_ok and host_ok else 1)
    return {"gpu_ingest_sigs_per_s": round(n_sig / ((ing + ver + comb) * 1e-3), 1),
            "gpu_ingest_ms": round(ing, 4), "gpu_ingest_verify_ms": round(ver, 4),
            "gpu_ingest_hbm_gbps": round(ing_bytes / (ing * 1e-3) / 1e9, 1), "gpu_ingest_bytes": ing_bytes,
            "gpu_ingest_parse_failures": int(len(pf)), "gpu_ingest_parse_failures_match_host": bool(host_pf_ok),
            "gpu_ingest_parity_mismatches": mism,
            "gpu_ingest_note": "raw payloads -> fd_txn_parse + signature-count scan + descriptor expansion on the "
                               "GPU, then verify + combine; isolated launches, HIP events"}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(arena, txns, sample, cpus):
    """The oracle (C restatement) on one pinned thread per physical core of
    this host (at most the GPU box's CPU share,
    workload.cpu_share_evidence), inputs statically
    partitioned.  Returns (baseline record, the CPU codes of the sample)."""
    from oracle import oracle as orc
    from firedancer_amd import workload
    sub = txns[:sample]
    t0 = time.perf_counter()
    codes = orc.verify_txns(arena, sub, cpus=cpus)
    dt = time.perf_counter() - t0
    rate = int(sub["sig_cnt"].sum()) / dt
    rec = {"value": round(rate, 1), "unit": "sigs/s", "cores": len(cpus), "kind": "port",
           "per_core": round(rate / len(cpus), 1), "cpu_model": cpu_model(), "cpus_pinned": cpus,
           "sample": f"first {len(sub)} txns of the rank-0 cfg1 batch, oracle/fd_ed25519_oracle.c "
                     f"(C restatement, radix-2^51, wNAF), one pinned thread per physical core on "
                     f"{len(cpus)} cores (the box's CPU share), {dt:.2f} s wall",
           "published_ref_per_core": "20-40K sigs/s/core (Icelake, book/guide/tuning.md:75) -- published, not measured",
           "cpu_share": workload.cpu_share_evidence()}
    return rec, codes


def adversarial(eng, n_txn, seed, ref_ms_per_sig, cpus):
    """SURVEY §8(d) / test_ed25519.c:920-951 bad-sig/msg modes at batch
    scale: 1M single-signature txns where EVERY signature fails the
    equation (one message bit flipped -> ERR_MSG), and where every R is
    corrupted (one bit of R -> decode failure or a wrong point).  Timed with
    HIP events like the headline's isolated launch; codes checked against
    the oracle on all txns."""
    from firedancer_amd import workload
    from oracle import oracle as orc
    out = {}
    for name, mode in (("eq_fail", workload.MODE_MSG), ("bad_r", workload.MODE_R)):
        arena, txns, _ = workload.make_txns(n_txn, seed, corrupt=1.0, corrupt_mode=mode)
        b = eng.upload(arena, txns)
        b.verify()
        got = b.codes()
        _, kv, kc = b.time(5)
        exp = orc.verify_txns(arena, txns, cpus=cpus)
        sigs_per_s = b.n_sig / ((kv + kc) * 1e-3)
        out[f"adv_{name}_sigs_per_s"] = round(sigs_per_s, 1)
        out[f"adv_{name}_vs_cfg2_isolated"] = round(ref_ms_per_sig / ((kv + kc) / b.n_sig), 4)   # throughput ratio
        out[f"adv_{name}_parity_mismatches"] = int((got != exp).sum())
        out[f"adv_{name}_codes"] = {int(c): int(k) for c, k in zip(*np.unique(exp, return_counts=True))}
        b.free()
    return out


# one verify = the launches of fdgpu_launch_verify_sigs (fdgpu_kernel_path():
# the half-size kernel + its full-length fallback, or the R-avoiding kernels),
# timed together with HIP events around the launches
VERIFY_KERNEL = "verify pipeline"


def pmc_traffic():
    """HBM bytes per verify-kernel launch from the newest committed PMC summary
    of the current kernel (profiles/rNN_pmc.json, tools/pmc_summary.py)."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "r[0-9][0-9]_pmc.json")), reverse=True):
        d = json.load(open(f))
        if d.get("kernel") == VERIFY_KERNEL:
            return d.get("hbm_bytes_per_launch"), os.path.basename(f)
    return None, None


def cfg3_rate(eng, eng_nobucket, cfg3):
    """BASELINE configs[2] (cfg3): 1-12 signatures sharing one message, msg up
    to the 1232-B MTU, 10% with one corrupted signature or message bit;
    device-resident, mean of HIP-event-timed verifies (secondary line, not
    `value`).  Timed with the signatures grouped by SHA-512 block count (the
    engine default) and in transaction order (FDGPU_FLAG_NO_BUCKET)."""
    arena, txns, modes = cfg3
    n_txn = len(txns)
    out = {}
    for tag, e in (("", eng), ("_unbucketed", eng_nobucket)):
        b = e.upload(arena, txns)
        b.verify()
        wall, kv, kc = b.time(5)
        n_sig = b.n_sig
        if not tag:
            codes = b.codes()
        else:
            out["cfg3_bucketing_codes_equal"] = bool((b.codes() == codes).all())
        b.free()
        out[f"cfg3{tag}_sigs_per_s"] = round(n_sig / ((kv + kc) * 1e-3), 1)
        out[f"cfg3{tag}_ms_per_batch"] = round(kv + kc, 3)
    out.update({"cfg3_txns": n_txn, "cfg3_sigs": n_sig,
                "cfg3_txns_per_s": round(n_txn / (out["cfg3_ms_per_batch"] * 1e-3), 1)})
    return out


def key_cache_rate(eng, device, n_txn, seed, pool=4096):
    """Signer reuse (a secondary line, not `value`): cfg1-shaped txns whose
    signers come from a pool of `pool` keys (10% corrupted, so ~1/30 of the
    keys are one-off corrupted ones), device-resident, timed without and with
    FDGPU_FLAG_KEY_CACHE (one A decode + table per distinct key); the two
    must give the same codes."""
    from firedancer_amd import VerifyEngine, workload
    arena, txns, modes = workload.make_txns(n_txn, seed, key_pool=pool)
    kc = VerifyEngine(device, max_txn=1024, ring_depth=1, key_cache=True)
    out, codes = {"keypool_txns": n_txn, "keypool_keys": pool}, {}
    for tag, e in (("", eng), ("_key_cache", kc)):
        b = e.upload(arena, txns)
        b.verify()
        codes[tag] = b.codes()
        _, kv, kcomb = b.time(5)
        out[f"keypool{tag}_sigs_per_s"] = round(b.n_sig / ((kv + kcomb) * 1e-3), 1)
        b.free()
    kc.close()
    out["keypool_key_cache_codes_equal"] = bool((codes[""] == codes["_key_cache"]).all())
    out["keypool_self_check"] = bool(((codes[""] == 0) == (modes == 0)).all())
    return out


def main():
    args = parse()
    dist = Dist()
    cpus = dist.cpus()
    from firedancer_amd import VerifyEngine, _lib, workload

    progress("generating the cfg1 batch", dist.rank)
    t_gen = time.perf_counter()
    arena, txns, modes = workload.cfg1(args.txns, seed=rank_seed(dist.rank))
    t_gen = time.perf_counter() - t_gen
    # the cfg5 tile lines first, in their child process, before this process
    # starts a HIP runtime or opens any engine: the tiles' 16+ slot streams
    # then have the device's hardware queues to themselves (with this
    # process's engines open beside them, one tile ran 34.5 M txn/s against
    # 38 M alone; profiles/r04/tile_run_order.md), and a rank and its child
    # are never two GPU processes at once
    cfg3 = workload.cfg3(args.cfg3_txns, seed=workload.CFG3_SEED + dist.rank) if args.cfg3_txns else None
    tl = None
    if args.tile and not args.no_extras:
        cfg3_tile = (workload.cfg3(args.tile_cfg3_txns, seed=workload.CFG3_SEED + 0x100 + dist.rank)
                     if args.tile_cfg3_txns else None)
        tl = tile_lines(dist.local_rank, arena, txns, modes, cpus, cfg3=cfg3_tile, world=dist.world)
        del cfg3_tile
        tl["tile_mux1_capacity_txns_per_s_node"] = round(dist.sum(tl["tile_mux1_capacity_txns_per_s"]), 1)
        tl["tile_published_ok_all_ranks"] = dist.sum(
            1 if all(v for k, v in tl.items() if k.endswith(("_published_ok", "_dedup_ok"))) else 0) == dist.world
        if dist.world > 1 and args.node_lines:   # the node's GPUs as one verify stage (before any rank starts HIP)
            dist.barrier()
            tl.update(node_lines(dist, arena, txns, modes, cpus, procs=args.node_procs or dist.world))
    # the engine library is loaded only now (loading the HIP runtime library
    # opens the driver: a rank holding it through its tile lines would be one
    # more GPU process beside its tile engines); a non-product build is refused
    progress("device-resident timed loop", dist.rank)
    build_info = _lib.require_product_build(allow_ab=args.ab_build)
    # one process per GPU; more ranks than visible GPUs (a rehearsal of the
    # multi-rank path on a one-GPU box) share devices round robin
    ndev = _lib.lib().fdgpu_device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no HIP device visible")
    device = dist.local_rank % ndev
    eng = VerifyEngine(device, max_txn=args.latency_batch, max_sig=2 * args.latency_batch,
                       max_arena=args.latency_batch * 1232, ring_depth=RING_DEPTH)
    # `queues` device-resident copies of the batch, each on its own HIP stream
    # + workspace: step i verifies copy i % queues, so consecutive 1M-signature
    # verifies overlap and the next one's waves fill the CUs the previous
    # one's partial last round leaves idle (every step is still a full verify)
    batches = [eng.upload(arena, txns) for _ in range(max(1, args.queues))]
    if args.queues > 1:
        for b in batches:
            b.own_queue()
    batch = batches[0]
    n_sig = batch.n_sig

    for i in range(max(args.warmup, len(batches))):
        batches[i % len(batches)].verify()
    eng.sync()
    self_check = all(bool(((b.codes() == 0) == (modes == 0)).all()) for b in batches)

    dist.barrier()
    eng.sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        batches[i % len(batches)].verify()
    eng.sync()
    dt = time.perf_counter() - t0
    dist.barrier()
    value, dt_max = aggregate(dist, n_sig, args.steps, dt)

    # live HIP-event timing of the verify pipeline (same stream, same batch)
    wall_ms, kv_ms, kc_ms = batch.time(max(3, min(args.steps, 10)))
    achieved = n_sig * MADS_PER_SIG / (kv_ms * 1e-3) / 1e12
    traffic, traffic_src = pmc_traffic()

    extras = {}
    if not args.no_extras:
        progress("latency and PCIe-inclusive legs", dist.rank)
        extras = latency_and_pcie(eng, arena, txns, args.latency_batch, args.latency_batches,
                                  pin_cpu=(cpus[1] if len(cpus) > 1 else cpus[0]) if cpus else None)
        extras.update(latency_frag_io(eng, arena, txns, batch.codes(), args.latency_batch, args.latency_batches,
                                      pin_cpu=(cpus[1] if len(cpus) > 1 else cpus[0]) if cpus else None))
        extras["latency_batch_txns"] = args.latency_batch
        if dist.rank == 0:
            progress("synchronous API", dist.rank)
            extras.update(sync_latency(arena, txns))
        if tl is not None:
            extras.update(tl)
        if args.cfg3_txns:
            progress("cfg3", dist.rank)
            eng_nb = VerifyEngine(device, max_txn=1024, ring_depth=1, bucket=False)
            extras.update(cfg3_rate(eng, eng_nb, cfg3))
            eng_nb.close()
        if tl is not None:
            # the tiles against this GPU's device-resident rate of the same txns (cfg1: one signature each)
            extras["tile_mux2_capacity_vs_device_resident"] = round(
                extras["tile_mux2_capacity_txns_per_s"] / (value / dist.world), 3)
            if "tile_mux2_capacity_cfg3_sigs_per_s" in extras:
                extras["tile_mux2_vs_mux1_capacity_cfg3"] = round(
                    extras["tile_mux2_capacity_cfg3_sigs_per_s"] / extras["tile_mux1_capacity_cfg3_sigs_per_s"], 3)
                if "cfg3_sigs_per_s" in extras:
                    extras["tile_mux2_capacity_cfg3_vs_device_resident"] = round(
                        extras["tile_mux2_capacity_cfg3_sigs_per_s"] / extras["cfg3_sigs_per_s"], 3)
        if args.keypool_txns:
            progress("key pool", dist.rank)
            extras.update(key_cache_rate(eng, device, args.keypool_txns, workload.CFG1_SEED + 0x700 + dist.rank))
        if args.host_fed:
            progress("host-fed 1M batches", dist.rank)
            extras.update(host_fed(device, arena, txns, n_sig, batch.codes(), value / dist.world,
                                   pin_cpu=(cpus[1] if len(cpus) > 1 else cpus[0]) if cpus else None))
        if args.adv_txns:
            progress("adversarial batches", dist.rank)
            extras.update(adversarial(eng, args.adv_txns, workload.CFG1_SEED + 0x400 + dist.rank,
                                      (kv_ms + kc_ms) / n_sig, cpus))
    cpu = None
    parity = {}
    if not args.no_extras:
        # full-size cfg2 parity: every GPU code of this rank's batch against the
        # oracle (rank 0 also times that oracle run as the CPU baseline)
        progress("parity against the oracle / CPU baseline", dist.rank)
        gpu_codes = batch.codes()
        n_chk = min(args.cpu_sample, len(txns))
        if dist.rank == 0 and dist.world == 1:
            cpu, cpu_codes = cpu_baseline(arena, txns, n_chk, cpus)
        else:
            from oracle import oracle as orc
            cpu_codes = orc.verify_txns(arena, txns[:n_chk], cpus=cpus)
        mism = int((gpu_codes[:n_chk] != cpu_codes).sum())
        parity = {"parity_checked_txns": int(dist.sum(n_chk)), "parity_mismatches": int(dist.sum(mism)),
                  "parity_codes": {int(c): int(k) for c, k in zip(*np.unique(cpu_codes, return_counts=True))}}
    if not args.no_extras:
        progress("GPU ingest", dist.rank)
        extras.update(gpu_ingest(eng, arena, txns, batch.codes()))
    for b in batches:
        b.free()
    eng.close()
    self_ok = dist.sum(1 if self_check else 0) == dist.world

    if dist.rank == 0:
        line = {
            "metric": "verified ed25519 sigs/sec (node)",
            "value": round(value, 1),
            "unit": "sigs/s",
            "n_gpus": dist.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded OpenSSL-signed Solana legacy txns, 10% one-bit corrupted)",
            "config": {"workload": f"cfg2: {args.txns} single-sig txns/GPU, msg U[180,220] B, 90% valid / 10% "
                                   "corrupted, device-resident batch, full verify + per-txn combine per step",
                       "sigs_per_gpu_per_step": n_sig, "parallelism": f"dp{dist.world} (independent per-GPU batches)",
                       "queues": len(batches)},
            "roofline": {"bound": "valu", "achieved": round(achieved, 3), "peak": round(VALU_MAD_PEAK_TOPS, 2),
                         "unit": "TOP/s", "frac": round(achieved / VALU_MAD_PEAK_TOPS, 4),
                         "traffic": traffic,
                         "peak_measured": VALU_MAD_MEASURED_TOPS,
                         "frac_measured": round(achieved / VALU_MAD_MEASURED_TOPS, 4),
                         "peak_note": "frac uses the nominal v_mad_u64_u32 issue peak (39.32 T/s); frac_measured "
                                      "the instruction's measured rate (33.88 T/s, profiles/r01_ubench_int.jsonl)",
                         "frac_overlapped": round(value / dist.world * MADS_PER_SIG / 1e12 / VALU_MAD_PEAK_TOPS, 4),
                         "note": f"INT32 v_mad_u64_u32 ops: {MADS_PER_SIG} algorithmic mads/sig x {n_sig} sigs / mean "
                                 f"{VERIFY_KERNEL} ({_lib.lib().fdgpu_kernel_path().decode()}) time "
                                 f"{kv_ms:.3f} ms (HIP events, compute stream); combine kernel "
                                 f"{kc_ms:.4f} ms; traffic source {traffic_src}"},
            "cpu_baseline": cpu,
            "self_check_codes": self_ok,
            "build": build_info,
            "gen_s": round(t_gen, 2),
        }
        line.update(parity)
        line.update(extras)
        print(json.dumps(line), flush=True)
    dist.close()
    # a parity failure fails the run (after the line is printed)
    if parity.get("parity_mismatches") or any(v for k, v in extras.items() if k.endswith("parity_mismatches")):
        sys.exit(3)


if __name__ == "__main__":
    main()
