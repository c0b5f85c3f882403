#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Usage: pmc_summary.py FETCH_DIR WRITE_DIR WORKLOAD [OUT_JSON]
Each DIR is a rocprofv3 -d directory written with --output-format csv.  Per the MI355X guide
(HBM section): FETCH_SIZE (KiB) reports half the bytes of a wide coalesced streaming read on
gfx950, so it is doubled; WRITE_SIZE is taken as is.  The result maps kernel -> mean bytes per
dispatch and is merged into OUT_JSON under WORKLOAD (bench.py reads
rollout_hbm_bytes_per_launch from profiles/pmc_traffic.json).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(lambda: [0.0, 0])
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "?")
                acc[name][0] += float(row["Counter_Value"])
                acc[name][1] += 1
    return {k: (v[0] / v[1], v[1]) for k, v in acc.items()}


def short(name):
    # the four-lane kernel's instantiations apart: <KIND, H, S, CEM, EXT, FM, KS> -- FM 1 the in-launch final
    # merge (2: with the sharded exchange), KS the step input as kernel argument (both: the host step's launch)
    if "rollout_quad_kernel<" in name:
        args = name.split("<", 1)[1].split(">")[0].replace(" ", "").split(",")
        fm = args[5] if len(args) > 5 else "0"
        tag = ({"1": "_fm", "true": "_fm", "2": "_fmx"}.get(fm, "")) + ("_ks" if len(args) > 6 and args[6] == "true" else "")
        return "rollout_quad_kernel" + tag
    if "rollout_kernel<" in name:  # <KIND, H, S, CEM, EXT, KS>
        args = name.split("<", 1)[1].split(">")[0].replace(" ", "").split(",")
        return "rollout_kernel" + ("_ks" if len(args) > 5 and args[5] == "true" else "")
    for key in ("rollout_quad_kernel", "rollout_kernel", "merge_kernel", "rng_kernel", "transpose_kernel",
                "advance_kernel", "tamols"):
        if key in name:
            return key
    return name[:60]


def main():
    fdir, wdir, workload = sys.argv[1:4]
    out = sys.argv[4] if len(sys.argv) > 4 else None
    fetch = per_kernel(fdir, "FETCH_SIZE")
    write = per_kernel(wdir, "WRITE_SIZE")
    kernels = {}
    for name in sorted(set(fetch) | set(write)):
        f, nf = fetch.get(name, (0.0, 0))
        w, nw = write.get(name, (0.0, 0))
        k = short(name)
        kernels[k] = {"fetch_bytes": 2 * f * 1024, "write_bytes": w * 1024, "dispatches": [nf, nw],
                      "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024}
    # the host step's rollout launch (fused next-step draws), as the bench's roofline times it
    roll = (kernels.get("rollout_quad_kernel_fm_ks") or kernels.get("rollout_quad_kernel_ks")
            or kernels.get("rollout_kernel_ks") or kernels.get("rollout_quad_kernel") or kernels.get("rollout_kernel"))
    res = {"kernels": kernels, "rollout_hbm_bytes_per_launch": roll["hbm_bytes_per_launch"] if roll else None,
           "note": "FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md HBM section) + WRITE_SIZE, KiB->bytes"}
    print(json.dumps(res, indent=1))
    if out:
        try:
            with open(out) as f:
                allres = json.load(f)
        except (OSError, ValueError):
            allres = {}
        allres[workload] = res
        with open(out, "w") as f:
            json.dump(allres, f, indent=1)


if __name__ == "__main__":
    main()
