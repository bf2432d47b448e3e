#!/usr/bin/env python3
"""Per-kernel PMC totals from rocprofv3 --pmc csv dirs.  Usage: tools/pmc_summary.py <dir>..."""
import collections
import csv
import glob
import re
import sys


def short(name):
    m = re.search(r"afm::\(anonymous namespace\)::([A-Za-z_0-9]+)", name)
    if m:
        return m.group(1)
    m = re.search(r"GLOBAL__N_1\d+([a-z_0-9]+?)(?:E|I)", name)
    if "afm" in name and m:
        return m.group(1)
    return name.split("(")[0][:40]


def templated(name):
    """short() plus the template arguments, so that instances of one template (the pooled and the
    per-date Grams) are reported apart."""
    k = short(name)
    m = re.search(re.escape(k) + r"(<[^()]*?>)\(", name)
    return k + m.group(1) if m else k


def main():
    for d in sys.argv[1:]:
      for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
          agg = collections.defaultdict(lambda: collections.defaultdict(float))
          disp = collections.defaultdict(set)
          for r in csv.DictReader(open(f)):
              k = templated(r["Kernel_Name"])     # zgram_kernel<7, 1, true> apart from <2, 0, false>
              agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
              disp[k].add(r["Dispatch_Id"])
          for k, v in agg.items():
              if "native" in k or "rocclr" in k or k.startswith("void"):
                  continue
              n = len(disp[k])
              print(f"{d.split('/')[-1]:6s} {k:30s} x{n}", " ".join(f"{c}={x / n:.4g}" for c, x in v.items()))


if __name__ == "__main__":
    main()
