"""Per-kernel timeline of the last bench step from a rocprofv3 kernel trace (start offset from the
step's first factor kernel, duration, stream).
Usage: python tools/trace_step.py run_kernel_trace.csv [factor launches per step (slabs), default 1]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
fk = [r for r in rows if "factor_panel" in r["Kernel_Name"]]
per = int(sys.argv[2]) if len(sys.argv) > 2 else 1
t0 = int(fk[-per]["Start_Timestamp"])
for r in rows:
    s = int(r["Start_Timestamp"])
    if s >= t0 - 2_000_000:
        name = r["Kernel_Name"].replace("afm::(anonymous namespace)::", "").replace("void ", "")
        print(f"{name[:34]:34s} start {(s - t0) / 1e6:8.3f}  dur {(int(r['End_Timestamp']) - s) / 1e6:7.3f}"
              f"  stream {r['Stream_Id']}  grid {r['Grid_Size_X']}x{r['Grid_Size_Y']}")
