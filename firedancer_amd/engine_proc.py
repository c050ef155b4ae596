"""The verify stage's GPU side as its own process (SURVEY.md §8(f) row 1,
"seccomp or separate engine process").

The reference's verify tile runs sandboxed: after privileged init only
write/fsync are allowed (src/app/fdctl/run/tiles/verify.seccomppolicy:1-19,
entered at src/disco/topo/fd_topo_run.c:96-103).  HIP needs ioctls on
/dev/kfd for every submission, so the batched verify tile (libfd_verify_tile
over the GPU engines) runs here, unsandboxed, in a process of its own that
joins the quic->verify and verify->dedup tango links in shared memory
(tile.Link.shm_create / fdt_link_new) -- the wiredancer arrangement
(src/wiredancer/c/wd_f1.h:71-112).  Tiles that only touch links (dedup, and
any other consumer) keep the reference's sandbox: tile.DedupTile.
fork_sandboxed / fdgpu_dtile_run_sandboxed.

    python -m firedancer_amd.engine_proc --in /dev/shm/quic_verify \\
        --out /dev/shm/verify_dedup --frags N [--gpus G]

prints the tile's final stats as one JSON line.
"""
import argparse
import json

from . import tile


def serve(in_path, out_path, verifier, frag_cnt, timeout_s=120.0, **tile_kw):
    """Join both links, run the verify tile until frag_cnt frags were seen on
    the in link and every batch is resolved; returns the tile's stats."""
    inl = tile.Link.shm_join(in_path)
    outl = tile.Link.shm_join(out_path)
    vt = tile.VerifyTile(inl, outl, verifier, **tile_kw)
    try:
        vt.run(frag_cnt, timeout_s=timeout_s)
        return vt.stats()
    finally:
        vt.close()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--in", dest="in_path", required=True)
    ap.add_argument("--out", dest="out_path", required=True)
    ap.add_argument("--frags", type=int, required=True)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--inflight", type=int, default=3)
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EEDF00D)
    ap.add_argument("--rr-idx", type=int, default=0)
    ap.add_argument("--rr-cnt", type=int, default=1)
    ap.add_argument("--flow-control", action="store_true")
    ap.add_argument("--timeout", type=float, default=120.0)
    a = ap.parse_args(argv)
    from . import VerifyEngine
    engines = [VerifyEngine(g, max_txn=a.batch, max_sig=a.batch * 12, max_arena=a.batch * 1232,
                            ring_depth=max(2, a.inflight)) for g in range(a.gpus)]
    ver = tile.EngineVerifier(engines)
    try:
        st = serve(a.in_path, a.out_path, ver, a.frags, timeout_s=a.timeout, hashmap_seed=a.seed,
                   batch_txn_max=a.batch, inflight_max=a.inflight, round_robin_idx=a.rr_idx,
                   round_robin_cnt=a.rr_cnt, flow_control=a.flow_control)
    finally:
        ver.close()
        for e in engines:
            e.close()
    print(json.dumps(st), flush=True)


if __name__ == "__main__":
    main()
