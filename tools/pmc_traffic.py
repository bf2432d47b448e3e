#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/prof_counters.sh).

Corrections (MI355X_MICROARCH.md, HBM section): both counters are in KiB; on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced streaming read, so it is doubled; WRITE_SIZE is taken
as is.  Output: JSON {kernel: {"fetch_bytes", "write_bytes", "hbm_bytes", "launches"}} per
launch (averaged over the launches of the profiled command), keyed by kernel name and by
kernel name + template arguments.

Usage: tools/pmc_traffic.py <pmc dir (with fetch/ and write/)> <out.json> [assets days]
(the bench workload the passes profiled; default 10000 5040)
"""
import collections
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short, templated  # noqa: E402


def per_launch(path, counter):
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            for k in {short(r["Kernel_Name"]), templated(r["Kernel_Name"])}:
                tot[k] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
    return {k: (tot[k] / len(disp[k]), len(disp[k])) for k in tot}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    wl = [int(x) for x in sys.argv[3:5]] if len(sys.argv) >= 5 else [10000, 5040]
    fetch = per_launch(os.path.join(src, "fetch"), "FETCH_SIZE")
    write = per_launch(os.path.join(src, "write"), "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        if "native" in k or "rocclr" in k or k.startswith("void"):
            continue
        fb = 2.0 * 1024.0 * fetch.get(k, (0.0, 0))[0]
        wb = 1024.0 * write.get(k, (0.0, 0))[0]
        out[k] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb,
                  "launches": max(fetch.get(k, (0, 0))[1], write.get(k, (0, 0))[1])}
    with open(dst, "w") as f:
        json.dump({"source": os.path.normpath(src), "workload": wl, "corrections": "FETCH_SIZE x2 (gfx950 "
                   "streaming-read undercount), KiB -> bytes", "kernels": out}, f, indent=1)


if __name__ == "__main__":
    main()
