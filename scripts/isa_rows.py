"""Static VALU instructions of one gca_alex_march.hip kernel instance by source line (ISA analysis; no GPU).
Compiles the R = 6 instances only (-DGCA_MARCH_ANALYSIS_R6) to device assembly with line info and counts, for the
instance named by its template flags, the VALU instructions attributed to each source line, largest first.
Usage: python scripts/isa_rows.py [OBS GROW NSEG FLATM] (default 0 0 1 2: the headline step, flat terrain + uniform layers)."""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gym-cellular-automata_amd", "csrc", "gca_alex_march.hip")


def main(obs=0, grow=0, nseg=1, flat=1, top=40):
    out = "/tmp/gca_march_r6.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-g", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                    "-munsafe-fp-atomics", "-DGCA_MARCH_ANALYSIS_R6", "--cuda-device-only", "-S", SRC, "-o", out],
                   check=True, stderr=subprocess.DEVNULL)
    L = open(out).read().split("\n")
    name = f"alex_march_kernelILi6ELb{obs}ELb{grow}ELi{nseg}ELi{flat}E"
    s = next(i for i, l in enumerate(L) if l.startswith("_Z") and name in l.split(":")[0])
    e = next(i for i in range(s, len(L)) if L[i].strip().startswith("s_endpgm"))
    files = {}
    for l in L:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
    cur, cnt, ops, tot = None, collections.Counter(), collections.Counter(), 0
    for l in L[s:e]:
        t = l.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if m:
            cur = (files.get(m.group(1), m.group(1)), int(m.group(2)))
            continue
        if t.startswith("v_"):
            cnt[cur] += 1
            ops[t.split()[0]] += 1
            tot += 1
    src = open(SRC).read().split("\n")
    print(f"{name}: {tot} VALU (static, whole kernel)")
    for (f, ln), v in cnt.most_common(top):
        text = src[ln - 1].strip()[:110] if f == os.path.basename(SRC) and ln else ""
        print(f"{v:5d}  {f}:{ln}  {text}")
    print(" ".join(f"{k}:{v}" for k, v in ops.most_common(25)))


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:5]] if len(sys.argv) >= 5 else [0, 0, 1, 2]
    main(*a)
