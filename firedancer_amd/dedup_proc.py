"""The dedup tile as a process of its own, inside the reference's sandbox
(src/app/fdctl/run/tiles/fd_dedup.c:89-205, dedup.seccomppolicy; entered
as fd_topo_run.c:96-103 enters it): joins the verify -> dedup links and its
dedup -> pack out link by path, then runs the tile in a forked child that
enters the seccomp policy first (fdgpu_dtile_run_sandboxed: only write to
fd 2 and exit remain).  This process never starts a HIP runtime, so the
fork is safe; it prints the child's final stats as one JSON line.

    python -m firedancer_amd.dedup_proc --in /dev/shm/verify_dedup_0 \\
        [--in ...] --out /dev/shm/dedup_pack --frags N [--idle-s 5]
"""
import argparse
import json
import os
import sys


def main(argv=None):
    from . import tile
    ap = argparse.ArgumentParser()
    ap.add_argument("--in", dest="in_paths", action="append", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--frags", type=int, required=True, help="stop once this many frags were consumed or lost")
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0xD5)
    ap.add_argument("--tcache-depth", type=int, default=4194302,
                    help="the reference's signature_cache_size (default.toml:910, fd_frankendancer.c:263)")
    ap.add_argument("--idle-s", type=float, default=10.0, help="stop after this long with no frag")
    ap.add_argument("--ready-file", default="", help="created once the sandboxed child runs")
    ap.add_argument("--cpu", type=int, default=-1, help="pin the tile to this CPU")
    ap.add_argument("--result", default="")
    ap.add_argument("--reliable", type=int, default=0,
                    help="1: write the tile's progress into each in link's fseq (its producers wait for it)")
    a = ap.parse_args(argv)
    if a.cpu >= 0:
        os.sched_setaffinity(0, {a.cpu})                 # the forked child keeps it
    ins = [tile.Link.shm_join(p) for p in a.in_paths]
    out = tile.Link.shm_join(a.out)
    dt = tile.DedupTile(ins, out, hashmap_seed=a.seed, tcache_depth=a.tcache_depth, reliable=bool(a.reliable))
    pid, stats = dt.fork_sandboxed(a.frags, idle_s=a.idle_s)
    if a.ready_file:
        open(a.ready_file, "w").close()
    _, status = os.waitpid(pid, 0)
    res = {"exit": os.WEXITSTATUS(status) if os.WIFEXITED(status) else -os.WTERMSIG(status), "stats": stats()}
    line = json.dumps(res)
    if a.result:
        with open(a.result + ".tmp", "w") as f:
            f.write(line + "\n")
        os.rename(a.result + ".tmp", a.result)
    print(line, flush=True)
    return 0 if res["exit"] in (0, 1) else 1


if __name__ == "__main__":
    sys.exit(main())
