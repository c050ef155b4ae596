"""Bring-up of the engine process's seccomp policy on a GPU box: the
cross-process pipeline (producer process -> engine processes -> sandboxed
dedup) with the engine processes in report mode (--sandbox 2: a call the
policy refuses fails with EPERM and is listed, nothing outside the policy
is carried out), then in enforce mode (--sandbox 1).  Prints one JSON line
per run: the refused syscalls, and whether every frag was published.

    python tools/sandbox_report.py [--txns 20000]
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

from firedancer_amd import workload  # noqa: E402
import xproc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=20000)
    ap.add_argument("--modes", default="2,1")
    a = ap.parse_args()
    arena, txns, modes = workload.cfg1(a.txns, seed=0x5A4D)
    ps = workload.payloads(arena, txns)
    pa, po, psz = workload.pack_payloads(ps)
    npz = os.path.join(tempfile.mkdtemp(prefix="fdgpu_sbx_"), "frags.npz")
    np.savez(npz, arena=pa, offs=po, sizes=psz)
    exp = int((modes == 0).sum())
    for mode in (int(x) for x in a.modes.split(",")):
        for procs in (1, 2):
            r = xproc.run(npz, len(ps), tiles=2, producers=2, mode="prefill", depth=1 << 16, batch=4096, inflight=4,
                          dedup=True, dedup_frags=2 * exp, engine_procs=procs, sandbox=mode, timeout=120)
            ers = r["engines"]
            print(json.dumps({"sandbox": mode, "engine_procs": procs,
                              "refused": [e.get("sandbox_refused") for e in ers],
                              "refused_calls": [e.get("sandbox_refused_calls") for e in ers],
                              "published": r["engine"]["stats"]["published"], "expected": 2 * exp,
                              "dedup_published": r["dedup"]["stats"]["published"],
                              "txns_per_s": r["txns_per_s"],
                              "stderr_refused": [ln for e in ers for ln in e.get("stderr_tail", "").splitlines()
                                                 if "refused" in ln]}), flush=True)


if __name__ == "__main__":
    main()
