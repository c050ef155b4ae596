"""Summarise rocprofv3 --pmc passes of the verify kernel into profiles/<tag>_pmc.json.

Usage: python tools/pmc_summary.py <tag> <dir_pass1> [<dir_pass2> ...]
(env PMC_OUT_DIR overrides the output directory, default profiles/)
Each dir holds one rocprofv3 `--pmc ... -o run --output-format csv` pass.
Reports per launch of the verify pipeline (KERNELS: the main verify kernel
and its tail kernels, summed; per-kernel medians kept): FETCH_SIZE / WRITE_SIZE (KB as
rocprofv3 reports them, and HBM bytes with the gfx950 FETCH_SIZE x2
correction of MI355X_MICROARCH.md §HBM), VALU instruction mix and busy
fractions.  The per-launch HBM bytes feed bench.py's roofline.traffic.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

PIPELINE = "verify pipeline"
# the launches of one fdgpu_launch_verify_sigs (half-size path, or the
# R-avoiding path of FDGPU_HALFSIZE=0 builds)
KERNELS = ("fdgpu_verify_hs_kernel", "fdgpu_full_kernel",
           "fdgpu_verify_ra_kernel", "fdgpu_tail_kernel", "fdgpu_finish_kernel", "fdgpu_fused_kernel")


def read_pass(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(lambda: defaultdict(list))      # kernel -> counter -> per-dispatch values
    meta = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = next((k for k in KERNELS if k in row.get("Kernel_Name", "")), None)
                if name is None:
                    continue
                vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
                if name in ("fdgpu_verify_hs_kernel", "fdgpu_verify_ra_kernel", "fdgpu_fused_kernel"):
                    meta = {k: row.get(k) for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size",
                                                    "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count") if k in row}
    return vals, meta


def main():
    tag, dirs = sys.argv[1], sys.argv[2:]
    per_kernel, meta = defaultdict(dict), {}
    for d in dirs:
        v, m = read_pass(d)
        meta.update(m)
        for kern, cs in v.items():
            for k, xs in cs.items():
                # several dispatches (warmup + steps): keep the median per launch
                xs = sorted(xs)
                per_kernel[kern][k] = xs[len(xs) // 2]
    agg = defaultdict(float)
    for cs in per_kernel.values():
        for k, x in cs.items():
            agg[k] += x
    agg = dict(agg)
    out = {"kernel": PIPELINE, "kernels": sorted(per_kernel), "counters_per_launch_median": agg,
           "per_kernel": per_kernel, "dispatch": meta}
    if "FETCH_SIZE" in agg:
        out["fetch_kb_reported"] = agg["FETCH_SIZE"]
        out["read_bytes_corrected"] = agg["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in agg:
        out["write_bytes"] = agg["WRITE_SIZE"] * 1024
    if "read_bytes_corrected" in out and "write_bytes" in out:
        out["hbm_bytes_per_launch"] = out["read_bytes_corrected"] + out["write_bytes"]
        out["hbm_bytes_per_launch_uncorrected"] = agg["FETCH_SIZE"] * 1024 + out["write_bytes"]
    if "SQ_INSTS_VALU" in agg and "SQ_INSTS_VALU_INT32" in agg:
        out["valu_int32_share"] = agg["SQ_INSTS_VALU_INT32"] / max(agg["SQ_INSTS_VALU"], 1)
    if "SQ_ACTIVE_INST_VALU" in agg and "SQ_WAVE_CYCLES" in agg:
        out["valu_active_per_wave_cycle"] = agg["SQ_ACTIVE_INST_VALU"] / max(agg["SQ_WAVE_CYCLES"], 1)
    out_dir = os.environ.get("PMC_OUT_DIR") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                           "profiles")
    path = os.path.join(out_dir, f"{tag}_pmc.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
