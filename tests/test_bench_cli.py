"""bench.py's helper plumbing on the CPU: the cfg5 tile lines run
tools/bench_tile.py in a child process with the command bench.tile_cmd
builds; it must parse with bench_tile's own parser and ask for every run of
bench.TILE_RUNS, or the driver's round-end bench dies in its tile leg on the
GPU box."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

import bench  # noqa: E402
import bench_tile  # noqa: E402


def test_tile_cmd_parses():
    cmd = bench.tile_cmd(0, [3, 4, 5, 6], "/tmp/x.npz", "/tmp/x.jsonl")
    assert cmd[1].endswith("tools/bench_tile.py")
    args = bench_tile.make_parser().parse_args(cmd[2:])
    assert args.mux == 1 and args.gpu_parse == 2 and args.producers_same_as_tiles == 1
    assert args.payload_npz == "/tmp/x.npz" and args.cpu_list == "3,4,5,6" and args.device_rank == 0
    assert args.hw_queues == bench.TILE_HW_QUEUES and args.reps == bench.TILE_REPS
    assert args.depth_lg == 21                                       # a prefill fits its links
    assert args.pair == bench.TILE_PAIR == 2                           # FDGPU_FLAG_PAIR_AUTO tile engines
    assert args.spread == bench.TILE_SPREAD == 2                       # FDGPU_FLAG_SPREAD_AUTO
    # paced runs: the reference's quic -> verify depth (receive_buffer_size, default.toml:888-893), and a
    # stream long enough that the producers can lap the tiles (>= 20 x the depth per link)
    assert args.depth_lg_paced == 14 and args.lap_guard == 1
    assert 1_000_000 * args.paced_reps // 4 >= 20 * (1 << args.depth_lg_paced)
    runs = [tuple(float(x) for x in r.split(",")) for r in args.sweep.split(";")]
    assert len(runs) == len(bench.TILE_RUNS)
    for (name, tiles_n, prods, rate), (t, b, k, r, p) in zip(bench.TILE_RUNS, runs):
        assert t == tiles_n and p == prods and r == rate and name
        assert (b, k) == (bench.TILE_BATCH, bench.TILE_INFLIGHT)
        assert rate > 0 or prods == tiles_n        # a prefilled run gives every link the whole stream


def test_tile_runs_shape():
    names = [r[0] for r in bench.TILE_RUNS]
    assert "mux1_capacity" in names and "mux2_capacity" in names      # the ratio line needs both
    for name, tiles_n, prods, rate in bench.TILE_RUNS:
        assert tiles_n >= 1 and prods >= 1 and (rate > 0 or rate == -1.0) and name


def test_tile_cmd_cfg3():
    cmd = bench.tile_cmd(1, [], "/tmp/y.npz", "/tmp/y.jsonl", bench.TILE_RUNS_CFG3, multi=1)
    args = bench_tile.make_parser().parse_args(cmd[2:])
    assert args.multi == 1 and args.device_rank == 1 and args.cpu_list == ""
    assert args.batch_sig_max == bench.TILE_CFG3_SIG_MAX
    assert len(args.sweep.split(";")) == len(bench.TILE_RUNS_CFG3)
    assert all(r[3] == -1.0 for r in bench.TILE_RUNS_CFG3)       # capacity lines
    # each run's signature cap (the sweep's sixth field): half-size batches when two tiles share the chip
    runs = [tuple(float(x) for x in r.split(",")) for r in args.sweep.split(";")]
    for (name, tiles_n, prods, rate), run in zip(bench.TILE_RUNS_CFG3, runs):
        assert len(run) == 6 and run[5] == bench.TILE_CFG3_SIG_MAX_BY_TILES[tiles_n]
    assert bench.TILE_CFG3_SIG_MAX_BY_TILES[2] <= bench.TILE_CFG3_SIG_MAX_BY_TILES[1] == bench.TILE_CFG3_SIG_MAX


def test_parent_rank_starts_no_hip_before_its_tile_child():
    """bench.py must not start a HIP runtime in a rank
    before that rank's tile child runs (8 ranks + 8 children would be 16 GPU
    processes beside the launcher); the child derives its device from the
    rank.  Checked on the source: no torch.cuda call anywhere, and the first
    device count comes after the tile lines."""
    src = open(os.path.join(REPO, "bench.py")).read()
    main = src[src.index("def main():"):]
    assert "torch.cuda" not in src
    # the engine library itself (libamdhip64 with it) is loaded only after the tile and node lines
    assert main.index("tile_lines(") < main.index("require_product_build(") < main.index("fdgpu_device_count()")
    assert main.index("node_lines(") < main.index("require_product_build(")
    assert "_lib.lib()" not in main[:main.index("require_product_build(")]
    assert main.index("fdgpu_device_count()") < main.index("VerifyEngine(")


def test_idle_first_counts_smt_siblings(monkeypatch):
    """bench.py pins tile and producer threads to the quietest cores
    (workload.idle_first); a core whose sibling hyperthread is busy counts
    as busy, so a core shared with another tenant goes last."""
    from firedancer_amd import workload
    ticks = iter([{0: 0, 1: 0, 2: 0, 3: 0, 128: 0, 129: 0, 130: 0, 131: 0},
                  {0: 5, 1: 0, 2: 0, 3: 1, 128: 0, 129: 90, 130: 0, 131: 0}])
    monkeypatch.setattr(workload, "_cpu_busy_ticks", lambda: next(ticks))
    monkeypatch.setattr(workload, "_smt_siblings", lambda c: [c, c + 128])
    monkeypatch.setattr("time.sleep", lambda s: None)
    assert workload.idle_first([0, 1, 2, 3]) == [2, 3, 0, 1]


def test_smt_siblings_of_this_host():
    from firedancer_amd import workload
    s = workload._smt_siblings(0)
    assert 0 in s and all(isinstance(c, int) for c in s)


def test_tile_cmd_xproc_runs():
    """The cross-process lines: every run of bench.TILE_RUNS_XPROC reaches
    bench_tile with its engine-process count and dedup switch (the sweep's
    seventh and eighth fields), among them two engine processes sharing the
    links and the e2e runs through the sandboxed dedup."""
    cmd = bench.tile_cmd(0, [3, 4, 5, 6, 7], "/tmp/z.npz", "/tmp/z.jsonl", bench.TILE_RUNS_XPROC, xproc=True)
    args = bench_tile.make_parser().parse_args(cmd[2:])
    assert args.xproc == 1 and args.reps == bench.TILE_REPS_XPROC
    assert args.dedup_depth == 4194302                  # the reference's signature_cache_size (default.toml:910)
    runs = [tuple(float(x) for x in r.split(",")) for r in args.sweep.split(";")]
    assert len(runs) == len(bench.TILE_RUNS_XPROC)
    seen = set()
    for (name, tiles_n, prods, rate, *rest), run in zip(bench.TILE_RUNS_XPROC, runs):
        assert run[:5] == (tiles_n, bench.TILE_BATCH, bench.TILE_INFLIGHT, rate, prods)
        if rest:
            procs, dedup = rest
            assert len(run) == 8 and run[6] == procs and run[7] == dedup and tiles_n % procs == 0
            seen.add((procs > 1, bool(dedup)))
        else:
            assert len(run) == 5
    assert (True, False) in seen and (False, True) in seen


def test_xproc_runs_per_world():
    """One rank of one: every cross-process line, two engine processes
    included; several ranks on a node: no line that starts two engine
    processes per rank (the node stays at one GPU process per GPU)."""
    assert bench.xproc_runs(1) == bench.TILE_RUNS_XPROC
    multi = bench.xproc_runs(8)
    assert multi and all(not (len(r) > 4 and r[4] > 1) for r in multi)
    assert any(len(r) > 5 and r[5] for r in multi)                 # the e2e dedup lines stay


def test_tile_child_streams_progress_and_parses(monkeypatch, capsys):
    """_tile_child echoes each of the child's lines to stderr as it comes (a
    long bench stays visibly alive; stdout keeps only the JSON line) and
    reads the runs back from the child's result file."""
    import json
    from firedancer_amd import workload
    arena, txns, modes = workload.cfg1(64, seed=1)
    runs = (("mux1_fake", 1, 1, 1e6),)
    n = len(runs) * bench.TILE_REPS

    def fake_cmd(rank, cpus, npz, out, runs, multi=0, xproc=False):
        row = dict(tiles=1, producers=1, txns_per_s=0.0, batch_latency_ms=dict(p50=1.0, p99=2.0), link_depth=16,
                   offered_txns_per_s=1e6, published_ok=True,
                   counters=dict(overrun=0, lapped=0, rescued=0, parse_fail=0, stall_max_ns=0, lap_margin_min=5))
        code = (f"import json\nrows = []\nprint('[bench_tile] ready', flush=True)\n"
                f"for i in range({n}):\n    r = dict({row!r}, txns_per_s=1.0 + i)\n"
                f"    print(json.dumps(r), flush=True)\n    rows.append(json.dumps(r))\n"
                f"open({out!r}, 'w').write(chr(10).join(rows) + chr(10))\n")
        return [sys.executable, "-c", code]

    monkeypatch.setattr(bench, "tile_cmd", fake_cmd)
    out = bench._tile_child(0, None, arena, txns, modes, runs)
    cap = capsys.readouterr()
    assert cap.out == ""
    assert cap.err.count("tile tiles 1 producers 1:") == n and "[bench_tile] ready" in cap.err
    assert out["tile_mux1_fake_txns_per_s_runs"] == [1.0 + i for i in range(n)]
    assert out["tile_mux1_fake_txns_per_s"] == sorted(out["tile_mux1_fake_txns_per_s_runs"])[n // 2]
    assert out["tile_mux1_fake_published_ok"] is True
    json.dumps(out)
