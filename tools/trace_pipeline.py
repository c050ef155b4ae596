"""Pipeline view of a rocprofv3 kernel trace (the gathered path): per kernel family, calls and mean
duration; over the busiest stretch, the time-averaged number of verify and
aux kernels running, and the verify sig-lanes those represent."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = []
fam = {}
for r in rows:
    n = r["Kernel_Name"]
    k = ("verify" if "verify" in n else "ingest" if "ingest" in n else "finish" if "finish_io" in n else
         "full" if "full_kernel" in n else "other")
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    fam.setdefault(k, []).append((s, e))
    ev.append((s, 1, k))
    ev.append((e, -1, k))
for k, v in fam.items():
    print(f"{k:7s} calls {len(v):5d} mean {sum(e - s for s, e in v) / len(v) / 1e3:8.1f} us")
vs = sorted(fam["verify"])
t0, t1 = vs[len(vs) // 10][0], vs[len(vs) * 9 // 10][0]          # middle 80% of the verify launches
ev.sort()
cur = {}
area = {}
last = t0
for t, d, k in ev:
    if t > t0:
        tt = min(t, t1)
        if tt > last:
            for kk, c in cur.items():
                area[kk] = area.get(kk, 0) + c * (tt - last)
            last = tt
    cur[k] = cur.get(k, 0) + d
span = t1 - t0
print(f"stretch {span / 1e6:.2f} ms, {sum(1 for s, e in vs if t0 <= s < t1)} verify launches")
for k, a in sorted(area.items()):
    print(f"  mean running {k:7s} {a / span:6.2f}")
