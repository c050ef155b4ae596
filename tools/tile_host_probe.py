"""Host-path scaling of the verify tile with no GPU: T step-loop tiles
(fdgpu_vtile, round-robin shares of one quic->verify link, as
fd_verify.c:46) over a verifier that accepts everything at once
(tools/null_verifier.c), fed by the line-rate producer thread.  Measures
what ingest + parse + tcache + publish cost per frag, and how it scales with
tile threads, apart from the engine.

    gcc -O2 -shared -fPIC -I include tools/null_verifier.c -o tools/libnullver.so
    python tools/tile_host_probe.py --tiles 1,2,4 --txns 1000000
"""
import argparse
import ctypes as c
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from firedancer_amd import tile, workload  # noqa: E402


class NullVerifier:
    sig_max = 1 << 30

    def __init__(self):
        lib = c.CDLL(os.path.join(REPO, "tools", "libnullver.so"))
        self.struct = tile.Verifier()
        lib.null_verifier_make(c.byref(self.struct))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="1,2,4")
    ap.add_argument("--txns", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--depth-lg", type=int, default=21)
    ap.add_argument("--prefill", type=int, default=0, help="1: publish everything before the tiles start")
    ap.add_argument("--mux", type=int, default=0, help="1: the mux-callback tile (fdgpu_vmux on fdt_mux_run)")
    ap.add_argument("--inflight", type=int, default=4)
    ap.add_argument("--gpu-parse", type=int, default=0, help="1 (with --mux 1): the tile hands the parse to the verifier")
    ap.add_argument("--cpus", default="", help="comma-separated CPUs for tile k (default: physical cores 1, 2, ...)"
                                               "; 'none' leaves the threads unpinned")
    args = ap.parse_args()
    topo = {}
    for cpu in sorted(os.sched_getaffinity(0)):
        b = f"/sys/devices/system/cpu/cpu{cpu}/topology/"
        try:
            topo[cpu] = tuple(open(b + f).read().strip() for f in ("physical_package_id", "die_id", "core_id"))
        except OSError:
            pass
    print(json.dumps({"affinity_topology(package,die,core)": topo}), flush=True)
    a, t, modes = workload.cfg1(args.txns, seed=0x5EED0005)
    ps = workload.payloads(a, t)
    arena, offs, sizes = workload.pack_payloads(ps)
    for T in [int(x) for x in args.tiles.split(",")]:
        inl = tile.Link(1 << args.depth_lg, 1232)
        vts = []
        for k in range(T):
            if args.mux:
                outl = tile.Link(1 << 14, tile.TPU_DCACHE_MTU,
                                 data_sz=tile.vmux_dcache_data_sz(1 << 14, args.batch, args.inflight))
                vts.append((tile.VerifyMuxTile(inl, outl, NullVerifier(), batch_txn_max=args.batch,
                                               inflight_max=args.inflight, round_robin_idx=k, round_robin_cnt=T,
                                               batch_bytes_max=args.batch * 2176, gpu_parse=bool(args.gpu_parse)),
                            outl))
            else:
                outl = tile.Link(1 << 12, tile.TPU_DCACHE_MTU)
                vts.append((tile.VerifyTile(inl, outl, NullVerifier(), batch_txn_max=args.batch,
                                            inflight_max=args.inflight, round_robin_idx=k, round_robin_cnt=T), outl))
        prod = None
        if args.prefill:
            prod = tile.Producer(inl, arena, offs, sizes, rate_tps=0)
            prod.join()
        cpus = [int(x) for x in args.cpus.split(",")] if args.cpus not in ("", "none") else \
            workload.physical_cpus()[1:] or [0]

        def body(vt, k):
            if args.cpus != "none":
                os.sched_setaffinity(0, {cpus[k % len(cpus)]})
            vt.run(len(ps), timeout_s=120)
            if args.mux:
                vt.mux_wall = time.perf_counter()
        ths = [threading.Thread(target=body, args=(vt, k)) for k, (vt, _) in enumerate(vts)]
        t0 = time.perf_counter()
        if not args.prefill:
            prod = tile.Producer(inl, arena, offs, sizes, rate_tps=0)
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        wall = time.perf_counter() - t0
        _, prod_s = prod.join() if not args.prefill else (None, 0.0)
        if args.mux:
            wall = max(vt.mux_wall for vt, _ in vts) - t0
        sts = [vt.stats() for vt, _ in vts]
        pub = sum(x["published"] for x in sts)
        print(json.dumps({"tiles": T, "txns": len(ps), "prefill": bool(args.prefill), "txns_per_s": round(len(ps) / wall, 1),
                          "wall_s": round(wall, 4), "producer_s": round(prod_s, 4), "published": pub,
                          "ns_per_frag_per_tile": round(wall * 1e9 / len(ps), 1),
                          "mux": bool(args.mux),
                          "ingest_ms_per_tile": [round(x["ingest_ns"] / 1e6, 1) for x in sts],
                          "submit_ms_per_tile": [round(x["submit_ns"] / 1e6, 1) for x in sts]}), flush=True)
        for vt, _ in vts:
            vt.close()


if __name__ == "__main__":
    main()
