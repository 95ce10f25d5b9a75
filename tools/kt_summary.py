"""Kernel / copy timeline of the LAST chain call in a rocprofv3 --kernel-trace CSV directory:
every kernel >= 0.05 ms from the first of the last K trellis_fwd_f64 launches on.
  python tools/kt_summary.py <dir with *_kernel_trace.csv> [K=#forward launches per call]"""
import csv
import glob
import sys

d = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = list(csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "trellis_fwd_f64" in r["Kernel_Name"]]
i0 = idx[-k]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0 - 2:]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    e = (int(r["End_Timestamp"]) - t0) / 1e6
    if e - s >= 0.05:
        print(f"{s:9.3f} {e:9.3f} {e - s:8.3f} {r['Kernel_Name'][:100]}")
