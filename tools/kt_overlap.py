"""For the last chain call in a rocprofv3 kernel trace: every forward / backtrack launch with its
duration and the other kernels (count, summed ms) running inside its span.
  python tools/kt_overlap.py <dir with *_kernel_trace.csv> <forward launches per call>"""
import collections
import csv
import glob
import sys

d, k = sys.argv[1], int(sys.argv[2])
rows = list(csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
fw = [e for e in ev if "trellis_fwd_f64" in e[2]]
t0 = fw[-k][0]
main = [e for e in ev if e[0] >= t0 and ("trellis_fwd_f64" in e[2] or "backtrack_f64" in e[2])]
for s, e, n in main:
    inside = collections.defaultdict(lambda: [0, 0.0])
    for s2, e2, n2 in ev:
        if s2 < e and e2 > s and (s2, e2, n2) != (s, e, n):
            key = n2.split("(")[0].split("<")[0].replace("void ", "").replace("cvk::", "")[-40:]
            inside[key][0] += 1
            inside[key][1] += (min(e, e2) - max(s, s2)) / 1e6
    print(f"{(s - t0) / 1e6:9.3f} {(e - s) / 1e6:8.3f} {n.split('(')[0][-50:]}")
    for key, (c, ms) in sorted(inside.items(), key=lambda x: -x[1][1]):
        print(f"{'':20s}{c:4d} x {key:40s} {ms:7.3f} ms inside")
last = max(e for s, e, n in ev)
print(f"last kernel ends {(last - t0) / 1e6:.3f} ms after the first forward's start")
