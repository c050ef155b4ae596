#!/bin/bash
# GPU-side ingest kernels under rocprofv3 (run on the GPU box via gpurun):
#   bash tools/ingest_measure.sh <tag>
# -> gpurun_out/<tag>/: probe.json (HIP-event split), trace/ (kernel trace + stats),
#    pmc_fetch/ and pmc_write/ (one counter pass each), ingest_summary.json
#    (per ingest kernel: mean duration, HBM bytes with the gfx950 FETCH_SIZE x2
#    correction, GB/s).
set -o pipefail
tag=$1
o=gpurun_out/$tag; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 240 python3 tools/ingest_probe.py > $o/probe.json 2> $o/probe.err || { tail $o/probe.err; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv \
  -- python3 tools/ingest_probe.py > $o/trace_probe.json 2> $o/trace.err || { tail $o/trace.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $o/pmc_fetch -o run --output-format csv \
  -- python3 tools/ingest_probe.py > $o/pmc_fetch.json 2> $o/pmc_fetch.err || { tail $o/pmc_fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $o/pmc_write -o run --output-format csv \
  -- python3 tools/ingest_probe.py > $o/pmc_write.json 2> $o/pmc_write.err || { tail $o/pmc_write.err; exit 1; }
python3 - $o <<'PY'
import csv, glob, json, os, sys
from collections import defaultdict
o = sys.argv[1]
K = ("fdgpu_frag_parse_kernel", "fdgpu_scan_local_kernel", "fdgpu_scan_blocks_kernel", "fdgpu_frag_expand_kernel",
     "fdgpu_frag_codes_kernel")
dur = defaultdict(list)
for f in glob.glob(os.path.join(o, "trace", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = next((k for k in K if k in r["Kernel_Name"]), None)
        if k:
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
ctr = defaultdict(lambda: defaultdict(list))
for d in ("pmc_fetch", "pmc_write"):
    for f in glob.glob(os.path.join(o, d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = next((k for k in K if k in r["Kernel_Name"]), None)
            if k:
                per[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, _, c), v in per.items():
            ctr[k][c].append(v)
med = lambda v: sorted(v)[len(v) // 2] if v else None
out = {"probe": json.load(open(os.path.join(o, "probe.json"))), "kernels": {}}
tot_ms = tot_b = 0.0
for k in K:
    ms = med(dur[k])
    fetch = med(ctr[k]["FETCH_SIZE"])
    write = med(ctr[k]["WRITE_SIZE"])
    hbm = (2 * fetch + write) * 1024 if fetch is not None and write is not None else None
    out["kernels"][k] = {"mean_ms": round(sum(dur[k]) / len(dur[k]), 5) if dur[k] else None, "median_ms": ms,
                         "launches": len(dur[k]), "fetch_kb": fetch, "write_kb": write, "hbm_bytes": hbm,
                         "hbm_gbps": round(hbm / (ms * 1e-3) / 1e9, 1) if hbm and ms else None}
    if ms and hbm:
        tot_ms += ms; tot_b += hbm
out["ingest_total"] = {"ms": round(tot_ms, 4), "hbm_bytes": tot_b, "hbm_gbps": round(tot_b / (tot_ms * 1e-3) / 1e9, 1) if tot_ms else None,
                       "note": "HBM bytes = 2 x FETCH_SIZE (gfx950 correction) + WRITE_SIZE, KB x 1024, medians per launch"}
json.dump(out, open(os.path.join(o, "ingest_summary.json"), "w"), indent=1)
print(json.dumps(out["ingest_total"]), json.dumps({k: (v["median_ms"], v["hbm_gbps"]) for k, v in out["kernels"].items()}))
PY
