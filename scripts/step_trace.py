#!/usr/bin/env python3
"""Per-step kernel sequence of host steps from a rocprofv3 kernel trace (measurement tool).

Usage: step_trace.py TRACE_CSV FIRST_KERNEL_SUBSTRING [SKIP]
Finds every launch whose name contains FIRST_KERNEL_SUBSTRING, takes the kernels up to the next such launch
as one step, and prints the median (us) of each kernel's duration and of the gaps between them, with names.
"""
import csv
import sys

import numpy as np


def main():
    fn, first = sys.argv[1], sys.argv[2]
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    rows = sorted(csv.DictReader(open(fn)), key=lambda r: int(r["Start_Timestamp"]))
    seq = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    starts = [i for i, s in enumerate(seq) if first in s[2]]
    steps = {}
    for a, b in zip(starts, starts[1:]):
        ks = seq[a:b]
        sig = tuple(k[2][:40] for k in ks)
        t = []
        for i, k in enumerate(ks):
            t.append((k[1] - k[0]) / 1000)
            t.append(((ks[i + 1][0] if i + 1 < len(ks) else seq[b][0]) - k[1]) / 1000)
        steps.setdefault(sig, []).append(t)
    for sig, ts in sorted(steps.items(), key=lambda x: -len(x[1])):
        if len(ts) < 5:
            continue
        m = np.median(np.array(ts[skip:] if len(ts) > skip + 5 else ts), axis=0)
        print(f"{len(ts)} steps of {len(sig)} kernels; total {m.sum():.2f} us")
        for i, nm in enumerate(sig):
            print(f"   {nm:42s} run {m[2 * i]:7.2f}  gap after {m[2 * i + 1]:7.2f}")


if __name__ == "__main__":
    main()
