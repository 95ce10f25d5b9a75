"""Every kernel >= MIN ms (default 0.05) of a rocprofv3 kernel trace from the LAST launch whose
name matches START_RE on (default the first kernel of the last call of a run: the last
`obs_first_bad`), with start / end relative to it.
  python tools/kt_list.py <dir with *_kernel_trace.csv> [START_RE] [MIN]"""
import csv
import glob
import re
import sys

d = sys.argv[1]
rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else "obs_first_bad")
mn = float(sys.argv[3]) if len(sys.argv) > 3 else 0.05
rows = list(csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
t0 = [e for e in ev if rx.search(e[2])][-1][0]
for s, e, n in ev:
    if s >= t0 and (e - s) / 1e6 >= mn:
        n = n.replace("void ", "").replace("cvk::", "").replace("(anonymous namespace)::", "")
        print(f"{(s - t0) / 1e6:9.3f} {(e - t0) / 1e6:9.3f} {(e - s) / 1e6:8.3f} {n[:110]}")
print(f"last end {(max(e for s, e, n in ev) - t0) / 1e6:.3f} ms")
