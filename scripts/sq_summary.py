#!/usr/bin/env python3
"""Per-kernel SQ counter means (per dispatch and per wave) from one rocprofv3 --pmc directory.

Usage: sq_summary.py PMC_DIR [OUT_JSON]
SQ_*_CYCLES count quad-cycles (MI355X_MICROARCH.md); a VALU instruction issues in one quad-cycle.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    name = name.replace("void ", "")
    return name.split("(")[0].replace("srbd::", "")


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else None
    acc = defaultdict(lambda: defaultdict(lambda: [0.0, 0]))
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                a = acc[short(row["Kernel_Name"])][row["Counter_Name"]]
                a[0] += float(row["Counter_Value"])
                a[1] += 1
    res = {}
    for k, cs in acc.items():
        m = {c: round(v[0] / v[1], 1) for c, v in cs.items()}
        w = m.get("SQ_WAVES") or 0
        if w and "SQ_INSTS_VALU" in m:
            m["per_wave"] = {
                "valu_insts": round(m["SQ_INSTS_VALU"] / w, 1),
                "wave_quad_cycles": round(m.get("SQ_WAVE_CYCLES", 0) / w, 1),
                "valu_active_frac": round(m.get("SQ_ACTIVE_INST_VALU", 0) / max(m.get("SQ_WAVE_CYCLES", 1), 1), 3),
                "wait_any_frac": round(m.get("SQ_WAIT_ANY", 0) / max(m.get("SQ_WAVE_CYCLES", 1), 1), 3),
                "wait_inst_any_frac": round(m.get("SQ_WAIT_INST_ANY", 0) / max(m.get("SQ_WAVE_CYCLES", 1), 1), 3),
            }
        res[k] = m
    res = {k: res[k] for k in sorted(res) if any(s in k for s in ("rollout", "merge", "rng", "copy16"))}
    print(json.dumps(res, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
