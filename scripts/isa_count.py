#!/usr/bin/env python3
"""Static instruction counts of the rollout kernels (gfx950 assembly of srbd_kernels.hip, no GPU).

Per horizon step = (instructions of the H=12 instantiation - those of H=10) / 2; also the whole
kernel's VGPR count and scratch size.  Usage: isa_count.py [--asm PATH] (default: compile to /tmp).
"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXTRA = [a for a in os.environ.get("ISA_FLAGS", "").split() if a]
SRC = os.path.join(ROOT, "quadruped-pympc-tamols_amd", "csrc", "srbd_kernels.hip")


def compile_asm(path):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", *EXTRA,
           "--cuda-device-only", "-S", "-o", path, SRC]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)


def functions(asm):
    lines = asm.split("\n")
    out, name, body = {}, None, []
    for l in lines:
        m = re.match(r"^(_Z\S+):", l)
        if m:
            name, body = m.group(1), []
            continue
        if name and l.startswith(".Lfunc_end"):
            out[name] = body
            name = None
            continue
        if name:
            t = l.strip()
            if t and not t.startswith((";", ".")) and not t.endswith(":"):
                body.append(t.split()[0])
    meta = {}
    for m in re.finditer(r"\.set (_Z\S+)\.(num_vgpr|private_seg_size), (\d+)", asm):
        meta.setdefault(m.group(1), {})[m.group(2)] = int(m.group(3))
    return out, meta


def mangled(kernel, kind, H, S, cem, ext):
    k = {"quad": "19rollout_quad_kernel", "thread": "14rollout_kernel"}[kernel]
    fm = "ELb0" if kernel == "quad" else ""  # the quad kernel's FM (in-launch final merge) flag
    return f"_ZN4srbd{k}ILi{kind}ELi{H}ELi{S}ELb{int(cem)}ELb{int(ext)}{fm}EEEvNS_10ModelConstEPKNS_9StepInputEPKfPfS7_iNS_6RngJobEiNS_9GroupArgsE"


def main():
    path = "/tmp/srbd_kernels_gfx950.s"
    if "--asm" in sys.argv:
        path = sys.argv[sys.argv.index("--asm") + 1]
    else:
        compile_asm(path)
    fns, meta = functions(open(path).read())
    for kernel in ("quad", "thread"):
        for kind, S in ((0, 0), (2, 2)):
            a, b = fns.get(mangled(kernel, kind, 12, S, kind == 2, False)), fns.get(mangled(kernel, kind, 16, S, kind == 2, False))
            if a is None or b is None:
                continue
            ca, cb = collections.Counter(a), collections.Counter(b)
            per = {k: (cb[k] - ca[k]) / 4 for k in set(ca) | set(cb)}
            valu = sum(v for k, v in per.items() if k.startswith("v_"))
            top = sorted(per.items(), key=lambda x: -x[1])[:12]
            m12 = meta.get(mangled(kernel, kind, 12, S, kind == 2, False), {})
            m16 = meta.get(mangled(kernel, kind, 16, S, kind == 2, False), {})
            print(f"{kernel} kind={kind}: per step {sum(per.values()):.1f} (VALU {valu:.1f}); H12 total {len(a)}; "
                  f"vgpr H12 {m12.get('num_vgpr')} H16 {m16.get('num_vgpr')} scratch {m12.get('private_seg_size')}/"
                  f"{m16.get('private_seg_size')}")
            print("   ", ", ".join(f"{k} {v:g}" for k, v in top))


if __name__ == "__main__":
    main()
