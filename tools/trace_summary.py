"""Reconcile a rocprofv3 kernel trace of bench.py's timed loop with its
ms_per_step (VERDICT r01 "the profile does not describe the timed
configuration").

Usage: python tools/trace_summary.py <trace_dir> <bench.json> [out.json]

bench.py verifies `queues` device-resident copies of the 1M-signature batch
round-robin, each on its own HIP stream, so consecutive steps overlap.  From
the per-dispatch start/end timestamps of the trace this reports, for the
verify pipeline (verify_ra + tail + finish + combine of one step):
  * each kernel's mean duration (what rocprofv3 --stats averages),
  * the span of the last `steps` pipelines (first start to last end) divided
    by `steps` -- the trace's own ms per step, to set beside bench's
    wall-clock ms_per_step,
  * how much of that span two pipelines run concurrently.
"""
import csv
import glob
import json
import os
import sys

PIPE = ("fdgpu_verify_ra_kernel", "fdgpu_tail_kernel", "fdgpu_finish_kernel", "fdgpu_combine_kernel")
PIPE_HS = ("fdgpu_verify_hs_kernel", "fdgpu_full_kernel", "fdgpu_combine_kernel")


def load(trace_dir):
    global PIPE
    f = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no kernel_trace.csv under {trace_dir}")
    rows = []
    recs = list(csv.DictReader(open(f[0])))
    if any(PIPE_HS[0] in r["Kernel_Name"] for r in recs):
        PIPE = PIPE_HS
    for r in recs:
        name = next((k for k in PIPE if k in r["Kernel_Name"]), None)
        if name:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name,
                         r.get("Queue_Id") or r.get("Stream_Id") or ""))
    rows.sort()
    return rows


def main():
    trace_dir, bench_json = sys.argv[1], sys.argv[2]
    bench = json.loads(open(bench_json).read().strip().splitlines()[-1])
    steps = int(bench["steps"])
    rows = load(trace_dir)
    ra = [r for r in rows if r[2] == PIPE[0]]
    per = {k: [(e - s) / 1e6 for s, e, n, _ in rows if n == k] for k in PIPE}
    last = PIPE[-1]
    # group each verify_ra launch with the tail/finish/combine that follow it
    # on the same queue
    pipes = []
    for s, e, n, q in ra:
        end = e
        for s2, e2, n2, q2 in rows:
            if q2 == q and s2 >= s and n2 != PIPE[0] and s2 < s + 60e6:
                if n2 == last:
                    end = max(end, e2)
                    break
                end = max(end, e2)
        pipes.append((s, end, q))
    # bench.py: max(warmup, queues) warm-up verifies, the `steps` timed ones,
    # then batch.time()'s max(3, min(steps, 10)) single-stream launches
    w = max(int(bench["warmup"]), int(bench["config"].get("queues") or 1))
    timed = pipes[w:w + steps]
    span = (max(e for _, e, _ in timed) - min(s for s, _, _ in timed)) / 1e6
    busy = 0.0
    ev = sorted([(s, 1) for s, _, _ in timed] + [(e, -1) for _, e, _ in timed])
    depth, last, conc = 0, None, 0.0
    for t, d in ev:
        if last is not None and depth >= 2:
            conc += (t - last) / 1e6
        if last is not None and depth >= 1:
            busy += (t - last) / 1e6
        depth += d
        last = t
    out = {
        "bench_ms_per_step": bench["ms_per_step"], "steps": steps, "queues": bench["config"].get("queues"),
        "trace_ms_per_step": round(span / steps, 4),
        "pipeline_ms_mean": round(sum((e - s) / 1e6 for s, e, _ in timed) / len(timed), 4),
        "kernel_ms_mean": {k: round(sum(v) / len(v), 4) for k, v in per.items() if v},
        "kernel_calls": {k: len(v) for k, v in per.items()},
        "span_ms": round(span, 3), "gpu_busy_ms": round(busy, 3), "two_pipelines_concurrent_ms": round(conc, 3),
        "queues_seen": sorted({q for _, _, q in timed}),
        "note": "trace_ms_per_step = span of the timed region's `steps` verify pipelines (after the warm-up ones) / "
                "steps; pipeline_ms_mean = one step's verify start to combine end (overlapping its neighbours when "
                "queues > 1); kernel_ms_mean covers every launch in the trace",
    }
    js = json.dumps(out, indent=1)
    print(js)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(js + "\n")


if __name__ == "__main__":
    main()
