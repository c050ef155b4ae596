"""N>1 path on CPU: two gloo ranks launched exactly like the driver launches
bench.py (torch.distributed.run, 127.0.0.1), independent shards, no
data-path collective, max-over-ranks timing."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_rank_gloo(tmp_path):
    out = str(tmp_path / "mr")
    env = dict(os.environ, MULTIRANK_OUT=out, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(REPO, "tests", "_multirank_worker.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = [json.load(open(f"{out}.{k}")) for k in range(2)]
    assert all(x["ok"] == 1 for x in res)
    assert res[0]["first"] != res[1]["first"]                  # distinct shards per rank
    assert res[0]["firsts_sum"] == res[0]["first"] + res[1]["first"]
    assert abs(res[0]["dt_max"] - res[1]["dt_max"]) < 1e-9     # both ranks agree on the max
    assert abs(res[0]["value"] - res[1]["value"]) < 1e-6
    assert res[0]["value"] > 0
    # ranks sharing one host affinity get disjoint physical cores (tile threads, oracle)
    assert res[0]["cpus"] and res[1]["cpus"]
    assert not set(res[0]["cpus"]) & set(res[1]["cpus"])
    # the node-level cfg5 lines: on rank 0 only, every frag through two engine processes and the dedup
    node = res[0]["node"]
    assert res[1]["node"] == {}
    for name, *_ in bench_runs():
        assert node[f"tile_{name}_published_ok"] and node[f"tile_{name}_dedup_ok"], (name, node)
        assert node[f"tile_{name}_overruns"] == 0 and node[f"tile_{name}_txns_per_s"] > 0
    assert "2 engine processes" in node["tile_node_config"]


def bench_runs():
    sys.path.insert(0, REPO)
    import bench
    return bench.NODE_RUNS
