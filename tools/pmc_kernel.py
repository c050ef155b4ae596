"""Per-launch PMC counters of one kernel from rocprofv3 counter_collection
CSVs: python tools/pmc_kernel.py <substring of kernel name> <csv>... -> JSON
{counter: mean per launch} (and launches)."""
import csv
import json
import sys

name, paths = sys.argv[1], sys.argv[2:]
acc, disp = {}, {}
for p in paths:
    for r in csv.DictReader(open(p)):
        if name not in r["Kernel_Name"]:
            continue
        acc.setdefault(r["Counter_Name"], {}).setdefault((p, r["Dispatch_Id"]), 0.0)
        acc[r["Counter_Name"]][(p, r["Dispatch_Id"])] += float(r["Counter_Value"])
out = {c: sum(v.values()) / len(v) for c, v in acc.items()}
out["launches"] = max(len(v) for v in acc.values()) if acc else 0
print(json.dumps(out, indent=1, sort_keys=True))
