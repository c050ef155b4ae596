"""Busy fraction of each CPU this process may run on, over a short window
(/proc/stat deltas): shows whether the cores a pinned tile would take are
shared with other work on the box.

    python tools/cpu_busy.py [--secs 0.5]
"""
import argparse
import json
import os
import time


def snap():
    out = {}
    for line in open("/proc/stat"):
        if line.startswith("cpu") and line[3].isdigit():
            f = line.split()
            v = list(map(int, f[1:]))
            out[int(f[0][3:])] = (sum(v), v[3] + v[4])          # total, idle + iowait
    return out


def busy(secs=0.5, cpus=None):
    cpus = sorted(cpus if cpus is not None else os.sched_getaffinity(0))
    a = snap()
    time.sleep(secs)
    b = snap()
    return {c: round(1 - (b[c][1] - a[c][1]) / max(1, b[c][0] - a[c][0]), 3) for c in cpus if c in a and c in b}


def idlest(n, secs=0.3, cpus=None):
    """The n least busy of `cpus` (default: this process's CPUs), least busy first."""
    b = busy(secs, cpus)
    return sorted(b, key=lambda c: (b[c], c))[:n]


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--secs", type=float, default=0.5)
    a = ap.parse_args()
    print(json.dumps({"loadavg": os.getloadavg(), "busy": busy(a.secs)}))
