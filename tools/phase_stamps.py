"""Per-phase cycle breakdown of fdgpu_verify_hs_kernel (diagnostic build).

    make -C firedancer_amd/csrc stamps
    FDGPU_LIB=build/stamps/libfd_ed25519_gpu.so python tools/phase_stamps.py [--txns N] [--out f.json]

Lane 0 of every wave stamps the shader clock at the phase boundaries of
fdgpu_kernels.hip (FDGPU_STAMP 0..7, fdgpu_stamps.h).  Reported: the mean
cycles each wave spends per phase (two waves share a SIMD, so a phase's
cycles include the time the partner wave held the VALU), the share of the
wave's lifetime, and the kernel's HIP-event time.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

PHASES = {"hs": ["sha512 + loads", "mod L + S check", "decode A + A table", "decode R + R table",
                 "lattice split + recode", "w = vS mod L + comb [w]B", "chain + check"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=1_000_000)
    ap.add_argument("--out", default=None)
    ap.add_argument("--path", choices=("hs",), default="hs", help="kernel path of the stamped build")
    args = ap.parse_args()
    import firedancer_amd as fa
    from firedancer_amd import _lib, workload
    L = _lib.lib()
    if not hasattr(L, "fdgpu_debug_stamps"):
        raise SystemExit("not a stamps build: set FDGPU_LIB=build/stamps/libfd_ed25519_gpu.so")
    L.fdgpu_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    arena, txns, modes = workload.cfg1(args.txns)
    eng = fa.VerifyEngine(0, max_txn=4096)
    b = eng.upload(arena, txns)
    b.verify()
    _, kv, kc = b.time(2)                       # the last of these verifies leaves its stamps
    n_waves = (b.n_sig + 63) // 64
    st = np.zeros(n_waves * 10, dtype=np.uint64)
    assert L.fdgpu_debug_stamps(st.ctypes.data, n_waves) == 0
    st = st.reshape(n_waves, 10).astype(np.int64)
    rt = st[:, 8:10]
    st = st[:, :8]
    d = np.diff(st, axis=1)
    ok = (d >= 0).all(axis=1)
    d = d[ok]
    life = (st[ok, 7] - st[ok, 0])
    # packing: how many waves are alive over the kernel's span, on the
    # constant 100-MHz clock (s_memrealtime; the shader clocks of the XCDs are
    # not aligned), in shader cycles at the clock the waves ran at
    clk = float(life.sum() / max((rt[ok, 1] - rt[ok, 0]).sum(), 1))   # shader cycles per 10 ns
    t0, t1 = (rt[ok, 0] * clk).astype(np.int64), (rt[ok, 1] * clk).astype(np.int64)
    span = float(t1.max() - t0.min())
    ev = np.concatenate([np.stack([t0, np.ones_like(t0)], 1), np.stack([t1, -np.ones_like(t1)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    alive = np.cumsum(ev[:, 1])
    dt = np.diff(ev[:, 0], append=ev[-1, 0])
    peak = int(alive.max())
    out = {"waves": int(n_waves), "waves_used": int(ok.sum()), "verify_ms": round(kv, 3),
           "wave_life_cycles_mean": round(float(life.mean()), 1),
           "wave_life_cycles_p01_p50_p99_max": [round(float(np.percentile(life, q)), 1) for q in (1, 50, 99, 100)],
           "span_cycles": span, "clock_ghz": round(clk / 10.0, 3), "span_ms": round(span / clk * 1e-5, 3),
           "alive_peak": peak, "alive_mean_over_span": round(float((alive * dt).sum() / max(span, 1.0)), 1),
           "span_below_90pct_peak": round(float(dt[alive < 0.9 * peak].sum() / max(span, 1.0)), 4),
           "phases": {p: {"cycles_mean": round(float(d[:, i].mean()), 1),
                          "share": round(float(d[:, i].mean() / life.mean()), 4)}
                      for i, p in enumerate(PHASES[args.path])},
           "note": "cycles per wave between FDGPU_STAMP boundaries (s_memtime, shader clock); 2 waves share a SIMD"}
    b.free()
    eng.close()
    js = json.dumps(out, indent=1)
    print(js)
    if args.out:
        open(args.out, "w").write(js + "\n")


if __name__ == "__main__":
    main()
