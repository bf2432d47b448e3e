#!/usr/bin/env python3
"""Loop census of one kernel in a gfx950 assembly file: every backward branch (a loop) with the
counts of its body's instructions -- f64 VALU, stores, scratch accesses, vmcnt waits.  Used to check
that the factor kernel's hot loops have no spill traffic and no store-draining waits.

    hipcc ... -S -o factors.s csrc/factors.hip   (or --save-temps)
    python tools/isa_loops.py factors.s factor_panel_kernelILi3ELb1 [min_f64]
"""
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    min_f64 = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + name + r"\w*:", l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, l in enumerate(body):
        m = re.match(r"\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            loops.append((labels[m.group(2)], i, m.group(2)))
    print(f"{name}: {len(body)} lines, {len(loops)} loops")
    for a, b, lab in loops:
        seg = [x.strip() for x in body[a:b + 1] if x.strip() and not x.strip().startswith(";")]
        f64 = sum(1 for x in seg if re.match(r"v_\w+_f64", x))
        if f64 < min_f64:
            continue
        valu = sum(1 for x in seg if x.startswith("v_"))
        st = sum(1 for x in seg if re.match(r"(global|buffer)_store", x))
        st16 = sum(1 for x in seg if re.match(r"(global|buffer)_store_dwordx4", x))
        scr = sum(1 for x in seg if x.startswith("scratch_") or re.match(r"buffer_\w+.*s\[0:3\]", x))
        vmw = [x for x in seg if re.match(r"s_waitcnt.*vmcnt", x)]
        perm = sum(1 for x in seg if "permlane" in x)
        print(f"  loop {lab} [{a}-{b}]: {len(seg)} instr, VALU {valu} (f64 {f64}, permlane {perm}), "
              f"stores {st} (16-B {st16}), scratch {scr}, vmcnt waits {len(vmw)} {vmw[:3]}")


if __name__ == "__main__":
    main()
