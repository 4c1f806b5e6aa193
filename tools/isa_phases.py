"""Dev probe: static instruction counts of k_dyn5 between its phase marks (a -DT1_ASM_MARKS device build turns every
T1_PROF_MARK into an assembly comment).  Counts follow the code layout: a region is the code from a mark to the next
mark in the listing, so it is exact for straight-line phases and indicative where branches interleave.

    python tools/isa_phases.py [--kernel-index 0] [extra hipcc flags]
"""
import collections
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    args = sys.argv[1:]
    ki = 0
    if args[:1] == ["--kernel-index"]:
        ki, args = int(args[1]), args[2:]
    out = "/tmp/isa_phases.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O1", "--offload-arch=gfx950", "-std=c++17", "-fno-slp-vectorize",
                    "--cuda-device-only", "-S", "-DT1_ASM_MARKS", *args, "-o", out,
                    os.path.join(REPO, "ti5_isaacgym_amd", "csrc", "t1env_dyn5.hip")], check=True)
    s = open(out).read().split("\n")
    starts = [k for k, l in enumerate(s) if re.match(r"^_Z\w+:", l)]
    ends = [k for k, l in enumerate(s) if l.startswith(".Lfunc_end")]
    i = starts[ki]
    j = [e for e in ends if e > i][0]
    print(s[i].split(":")[0][:60])
    cur, regions = "entry", []
    c = collections.Counter()
    for l in s[i:j]:
        t = l.strip()
        m = re.search(r";@@MARK (\S+)", t)
        if m:
            regions.append((cur, c))
            cur, c = m.group(1), collections.Counter()
            continue
        if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
            continue
        op = t.split()[0]
        cat = ("acc" if op.startswith("v_accvgpr") else "lane" if op.startswith(("v_readlane", "v_writelane"))
               else "valu" if op.startswith("v_") else "lds" if op.startswith("ds_") else
               "smem" if op.startswith(("s_load", "s_buffer")) else "wait" if op == "s_waitcnt" else
               "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "salu")
        c[cat] += 1
    regions.append((cur, c))
    for name, c in regions:
        if sum(c.values()):
            print(f"after mark {name:>6s}: total {sum(c.values()):6d}  " +
                  "  ".join(f"{k} {c[k]}" for k in ("valu", "salu", "lds", "smem", "vmem", "wait", "acc", "lane")))


if __name__ == "__main__":
    main()
