#!/usr/bin/env python3
"""HBM bytes of a whole multi-launch pass (config D: the factor build by time slab) from the
rocprofv3 FETCH_SIZE / WRITE_SIZE passes of tools/gpu_pmc_config_d.sh.  Sums every dispatch of the
named kernels and divides by the number of passes the profiled command ran.  Corrections as in
tools/pmc_traffic.py (MI355X_MICROARCH.md: FETCH_SIZE x2, KiB -> bytes).

Usage: tools/pmc_pass.py <pmc dir (fetch/, write/)> <out.json> <passes> <assets> <bars> kernel...
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def totals(path, counter, names):
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if r["Counter_Name"] == counter and k in names:
                tot[k] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
    return tot, {k: len(v) for k, v in disp.items()}


def main():
    src, dst, passes = sys.argv[1], sys.argv[2], int(sys.argv[3])
    wl = [int(sys.argv[4]), int(sys.argv[5])]
    names = set(sys.argv[6:])
    f, nf = totals(os.path.join(src, "fetch"), "FETCH_SIZE", names)
    w, nw = totals(os.path.join(src, "write"), "WRITE_SIZE", names)
    ks = {}
    for k in sorted(names):
        fb = 2.0 * 1024.0 * f.get(k, 0.0) / passes
        wb = 1024.0 * w.get(k, 0.0) / passes
        ks[k] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb,
                 "launches_per_pass": max(nf.get(k, 0), nw.get(k, 0)) / passes}
    out = {"source": os.path.normpath(src), "workload": wl, "passes": passes,
           "corrections": "FETCH_SIZE x2 (gfx950 streaming-read undercount), KiB -> bytes",
           "kernels": ks, "hbm_bytes_per_pass": sum(v["hbm_bytes"] for v in ks.values())}
    with open(dst, "w") as fo:
        json.dump(out, fo, indent=1)
    print(json.dumps(out)[:600])


if __name__ == "__main__":
    main()
