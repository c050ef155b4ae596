"""Per-CPU speed and clock probe of a GPU box's host (CPU only): a fixed
integer loop pinned to each of the first N CPUs of the affinity mask, timed
with perf_counter, plus the clock's resolution -- to pick cores for the tile
threads that no other tenant is using.  Prints one JSON line."""
import json
import os
import sys
import time


def spin(n=3_000_000):
    x = 0
    for i in range(n):
        x = (x * 1103515245 + i) & 0xFFFFFFFF
    return x


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    cpus = sorted(os.sched_getaffinity(0))[:n]
    res = {}
    keep = os.sched_getaffinity(0)
    for c in cpus:
        os.sched_setaffinity(0, {c})
        t0 = time.perf_counter()
        spin()
        res[c] = round((time.perf_counter() - t0) * 1e3, 1)
    os.sched_setaffinity(0, keep)
    ts = [time.perf_counter_ns() for _ in range(100000)]
    d = [b - a for a, b in zip(ts, ts[1:]) if b > a]
    topo = {}
    for c in cpus:
        b = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            topo[c] = [open(b + f).read().strip() for f in ("physical_package_id", "die_id", "core_id")]
        except OSError:
            pass
    print(json.dumps({"spin_ms_by_cpu": res, "clock_min_step_ns": min(d) if d else None,
                      "load": open("/proc/loadavg").read().strip(), "topology": topo}))


if __name__ == "__main__":
    main()
