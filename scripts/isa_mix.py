#!/usr/bin/env python3
"""Static instruction mix of one kernel instantiation (gfx950 assembly, no GPU).

Usage: isa_mix.py [--src FILE] [--flags "..."] [--top N] [--dump OUT.s] NAME_REGEX
Compiles the source (default csrc/srbd_kernels.hip) to assembly and prints, for every kernel whose mangled
name matches NAME_REGEX: instruction count, VALU count, branches, scalar waits, VGPRs, scratch, top opcodes.
"""
import argparse
import collections
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "quadruped-pympc-tamols_amd", "csrc")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--src", default="srbd_kernels.hip")
    ap.add_argument("--flags", default="")
    ap.add_argument("--top", type=int, default=24)
    ap.add_argument("--dump", default=None)
    a = ap.parse_args()
    out = "/tmp/isa_mix_%d.s" % os.getpid()
    extra = ["-fno-slp-vectorize"] if a.src == "srbd_rollout_thread.hip" else []
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    *extra, *a.flags.split(), "--cuda-device-only", "-S", "-o", out, os.path.join(CSRC, a.src)],
                   check=True, stderr=subprocess.DEVNULL)
    asm = open(out).read()
    os.unlink(out)
    for m in re.finditer(r"^(_Z\S+):", asm, re.M):
        name = m.group(1)
        if not re.search(a.name, name):
            continue
        end = asm.index(".Lfunc_end", m.end())
        body = [l.strip() for l in asm[m.end():end].split("\n")]
        ins = [l.split()[0] for l in body if l and not l.startswith((";", ".")) and not l.endswith(":")]
        c = collections.Counter(ins)
        meta = {k: int(v) for k, v in re.findall(r"\.set " + re.escape(name) + r"\.(num_vgpr|private_seg_size|numbered_sgpr), (\d+)", asm)}
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        br = sum(v for k, v in c.items() if k.startswith("s_cbranch"))
        print(f"{name[:110]}\n  insts {len(ins)}  VALU {valu}  branches {br}  lgkm-waits "
              f"{sum(1 for l in body if l.startswith('s_waitcnt lgkmcnt(0)'))}  {meta}")
        print("  " + ", ".join(f"{k} {v}" for k, v in c.most_common(a.top)))
        if a.dump:
            open(a.dump, "w").write("\n".join(body))


if __name__ == "__main__":
    main()
