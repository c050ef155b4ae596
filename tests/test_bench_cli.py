"""bench.py's helper plumbing on the CPU: the cfg5 tile lines hand
bench_tile.run_once_mux an options namespace built by bench.tile_args; every
option run_once_mux (and the start_producer it calls) reads must be there, or
the driver's round-end bench dies in its tile leg on the GPU box."""
import ast
import inspect
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

import bench  # noqa: E402
import bench_tile  # noqa: E402


def _args_read(fn):
    """attribute names read as args.X (getattr(args, "X", default) excluded)"""
    tree = ast.parse(inspect.getsource(fn))
    return {n.attr for n in ast.walk(tree)
            if isinstance(n, ast.Attribute) and isinstance(n.value, ast.Name) and n.value.id == "args"}


def test_tile_args_cover_run_once_mux():
    need = _args_read(bench_tile.run_once_mux) | _args_read(bench_tile.start_producer)
    for prods, rate in ((1, 0.0), (2, 16e6)):
        ns = bench.tile_args(prods, rate)
        missing = sorted(a for a in need if not hasattr(ns, a))
        assert not missing, f"bench.tile_args lacks {missing}"


def test_tile_runs_shape():
    for name, tiles_n, prods, rate in bench.TILE_RUNS:
        assert tiles_n >= 1 and prods >= 1 and (rate > 0 or rate == -1.0) and name
        assert bench.tile_args(prods, rate).depth_lg == (21 if rate < 0 else 19)   # a prefill fits its links
