"""Timeline of the last call in a rocprofv3 --kernel-trace [--memory-copy-trace] csv directory.

  python tools/trace_timeline.py <trace dir> <kernel-name substring marking the call's start> [k]

Prints every kernel dispatch and copy from the LAST (k = -1, or the k-th from the end) dispatch
whose name contains the marker on,
in start order, in ms relative to that dispatch, with the gap after the previous item's end.
"""
import csv
import glob
import os
import sys


def main():
    d, marker = sys.argv[1], sys.argv[2]
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:100]))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         "COPY " + r.get("Direction", "") + " " + r.get("Size", "")))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if marker in r[2]]
    if not starts:
        raise SystemExit(f"no dispatch matches {marker!r}")
    i0 = starts[int(sys.argv[3]) if len(sys.argv) > 3 else -1]
    t0 = rows[i0][0]
    prev = None
    for s, e, k in rows[i0:]:
        gap = "" if prev is None else f" (+{(s - prev) / 1e6:.3f} after prev end)"
        print(f"{(s - t0) / 1e6:9.3f} -> {(e - t0) / 1e6:9.3f} ms ({(e - s) / 1e6:8.3f}) {k}{gap}")
        prev = max(prev or 0, e)


if __name__ == "__main__":
    main()
