"""Writes bench.py's tile-line payload file (arena, offs, sizes, modes, n_sig)
for standalone tools/bench_tile.py runs: the rank-0 cfg1 (or --multi 1: cfg3)
batch as raw wire payloads."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import workload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--txns", type=int, default=1_000_000)
ap.add_argument("--multi", type=int, default=0)
ap.add_argument("--out", required=True)
a = ap.parse_args()
arena, txns, modes = (workload.cfg3(a.txns, seed=workload.CFG3_SEED) if a.multi else
                      workload.cfg1(a.txns, seed=workload.CFG1_SEED))
pa, po, ps = workload.pack_payloads(workload.payloads(arena, txns))
np.savez(a.out, arena=pa, offs=po, sizes=ps, modes=modes, n_sig=int(txns["sig_cnt"].sum()))
print(a.out, len(po))
