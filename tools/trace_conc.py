"""Kernel concurrency of a rocprofv3 kernel trace (run_kernel_trace.csv):
the dense stretches of verify launches (split at gaps > 5 ms), how many
kernels ran at once for what fraction of each stretch, the verify launches'
durations and their grid items per second.  Used on the two-tile mux runs
(tools/gpu_run_r03l.sh) to see whether the GPU or the tiles bound them.

    python3 tools/trace_conc.py gpurun_out/r03l/trace/run_kernel_trace.csv
"""
import csv
import statistics
import sys


def conc_hist(ks):
    ev = sorted([(s, 1) for s, e, *_ in ks] + [(e, -1) for s, e, *_ in ks])
    c, last, out = 0, None, {}
    for t, x in ev:
        if last is not None:
            out[c] = out.get(c, 0) + (t - last)
        c += x
        last = t
    tot = sum(out.values()) or 1
    return {k: round(v / tot, 3) for k, v in sorted(out.items())}


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_X"]))
                for r in rows)
    v = [k for k in ks if "verify_hs" in k[2]]
    starts = [k[0] for k in v]
    cut = [i for i, (a, b) in enumerate(zip(starts, starts[1:])) if b - a > 5_000_000]
    prev = 0
    for i in cut + [len(v) - 1]:
        a, b = prev, i
        prev = i + 1
        if b - a < 20:
            continue
        t0, t1 = v[a][0], v[b][1]
        sub = [k for k in ks if k[0] >= t0 and k[1] <= t1]
        items = sum(k[3] for k in v[a:b + 1])
        dur = [(k[1] - k[0]) / 1e3 for k in v[a:b + 1]]
        print(f"stretch: {b - a + 1} verify launches in {(t1 - t0) / 1e6:.2f} ms, "
              f"{items} grid items ({items / (t1 - t0) * 1e3:.1f} M/s)")
        print(f"  verify duration us p10/p50/p90: {sorted(dur)[len(dur) // 10]:.0f} / "
              f"{statistics.median(dur):.0f} / {sorted(dur)[9 * len(dur) // 10]:.0f}")
        print(f"  kernels running at once (fraction of the stretch): {conc_hist(sub)}")
        print(f"  verify launches at once: {conc_hist(v[a:b + 1])}")


if __name__ == "__main__":
    main(sys.argv[1])
