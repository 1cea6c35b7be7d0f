#!/usr/bin/env python3
"""List the scratch spills / reloads of each kernel in a gfx950 .s file and whether they sit inside the kernel's
largest loop (the marching row loop). Usage: python scripts/spills.py file.s [name-filter]"""
import re
import sys

def loop_mix(path, filt):
    """instruction mix (VALU / SALU / LDS / VMEM) inside the largest loop of the first kernel matching filt"""
    src = open(path).read().split("\n")
    starts = [i for i, l in enumerate(src) if re.match(r"^_Z\S*:", l)]
    for n, st in enumerate(starts):
        if filt not in src[st]:
            continue
        end = starts[n + 1] if n + 1 < len(starts) else len(src)
        body = src[st:end]
        best = None
        for i, l in enumerate(body):
            m = re.match(r"^\.(LBB\d+_\d+):.*Loop Header", l)
            if m:
                back = max((j for j, x in enumerate(body) if re.search(r"s_(c?branch\w*) \.%s$" % m.group(1), x)), default=i)
                if best is None or back - i > best[1] - best[0]:
                    best = (i, back)
        mix = {"v_": 0, "s_": 0, "ds_": 0, "global_": 0, "buffer_": 0, "scratch_": 0}
        for l in body[best[0]:best[1] + 1]:
            t = l.strip().split(" ")[0]
            for k in mix:
                if t.startswith(k):
                    mix[k] += 1
        return mix


def main():
    src = open(sys.argv[1]).read().split("\n")
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    starts = [i for i, l in enumerate(src) if re.match(r"^_Z\S*:", l)]
    for n, st in enumerate(starts):
        name = src[st].split(":")[0]
        if filt not in name:
            continue
        end = starts[n + 1] if n + 1 < len(starts) else len(src)
        body = src[st:end]
        loops = {}
        for i, l in enumerate(body):
            m = re.match(r"^\.(LBB\d+_\d+):.*Loop Header", l)
            if m:
                lab = m.group(1)
                back = max((j for j, x in enumerate(body) if re.search(r"s_(c?branch\w*) \.%s$" % lab, x)), default=i)
                loops[lab] = (i, back)
        big = max(loops.items(), key=lambda kv: kv[1][1] - kv[1][0]) if loops else None
        sc = [(i, l.strip().split(";")[0].strip()) for i, l in enumerate(body) if "scratch_" in l]
        inl = [x for x in sc if big and big[1][0] <= x[0] <= big[1][1]]
        print(f"{name[:70]}: loop {big[1] if big else None} ({big[1][1]-big[1][0] if big else 0} lines), "
              f"{len(sc)} scratch ops, {len(inl)} in the loop")
        for i, l in inl:
            print(f"    {i}: {l}")


if __name__ == "__main__":
    main()
