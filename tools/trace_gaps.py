"""Timeline of one rocprofv3 --kernel-trace CSV: per-kernel spans (in dispatch order) and the
device-idle gaps between them, for the last `--last` ms of the trace (the final timed call).
Usage: python tools/trace_gaps.py <kernel_trace.csv> [--window-ms W]"""
import csv
import sys

path = sys.argv[1]
win = float(sys.argv[sys.argv.index("--window-ms") + 1]) if "--window-ms" in sys.argv else 400.0
rows = []
for r in csv.DictReader(open(path)):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70], r.get("Queue_Id", "")))
rows.sort()
t_end = max(e for _, e, _, _ in rows)
rows = [r for r in rows if r[1] >= t_end - win * 1e6]
t0 = rows[0][0]
busy_until = t0
idle = 0.0
for s, e, n, q in rows:
    gap = (s - busy_until) / 1e6
    if gap > 0.05:
        print(f"   idle {gap:8.3f} ms")
        idle += gap
    print(f"{(s - t0) / 1e6:9.3f} -> {(e - t0) / 1e6:9.3f} ms ({(e - s) / 1e6:8.3f}) q{q} {n}")
    busy_until = max(busy_until, e)
print(f"span {(busy_until - t0) / 1e6:.3f} ms, device idle {idle:.3f} ms")
