"""Per-kernel durations and the gaps between consecutive dispatches from a rocprofv3
--kernel-trace CSV (kernel_trace.csv): python tools/trace_gaps.py <dir> [kernel regex]"""
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
sel = [(s, e, k) for s, e, k in rows if rx.search(k)]
if not sel:
    sys.exit("no kernels matched")
dur = [e - s for s, e, _ in sel]
gaps = [sel[i + 1][0] - sel[i][1] for i in range(len(sel) - 1)]
gaps.sort()
print(f"{len(sel)} dispatches of /{rx.pattern}/: mean duration {sum(dur) / len(dur) / 1e3:.2f} us, "
      f"median gap {gaps[len(gaps) // 2] / 1e3 if gaps else 0:.2f} us, p90 gap {gaps[int(len(gaps) * 0.9)] / 1e3 if gaps else 0:.2f} us")
names = sorted({k for _, _, k in sel})
for n in names[:6]:
    dd = [e - s for s, e, k in sel if k == n]
    print(f"  {len(dd):6d} x {sum(dd) / len(dd) / 1e3:9.2f} us  {n[:110]}")
