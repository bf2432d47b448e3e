#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (results .db or kernel_trace.csv) per kernel:
calls, average / total duration.  Usage: tools/rocprof_summary.py <db-or-csv-or-dir> [out.md]"""
import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def from_db(path):
    c = sqlite3.connect(path)
    q = ("select s.kernel_name, d.end - d.start from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    return list(c.execute(q))


def from_csv(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return rows


def main():
    src = sys.argv[1]
    if os.path.isdir(src):
        cands = glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True) or \
            glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
        src = cands[0]
    rows = from_db(src) if src.endswith(".db") else from_csv(src)
    agg = defaultdict(list)
    for name, ns in rows:
        agg[name].append(ns)
    tot = sum(sum(v) for v in agg.values())
    lines = [f"source: {os.path.basename(src)}", "",
             "| kernel | calls | avg ms | total ms | % |", "|---|---:|---:|---:|---:|"]
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        short = name.replace("(anonymous namespace)::", "").split("(")[0]
        if short.startswith("_ZN3afm"):
            short = short.replace("_ZN3afm12_GLOBAL__N_1", "afm::")
        lines.append(f"| {short[:80]} | {len(v)} | {sum(v) / len(v) / 1e6:.3f} | "
                     f"{sum(v) / 1e6:.2f} | {100 * sum(v) / tot:.1f} |")
    text = "\n".join(lines) + "\n"
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
