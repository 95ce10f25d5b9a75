"""Per-launch HBM bytes of the forward trellis kernel from rocprofv3 --pmc CSVs.

FETCH_SIZE / WRITE_SIZE are kilobytes (TCC EA request counters).  Per MI355X_MICROARCH.md
§HBM: on gfx950 FETCH_SIZE reads exactly half the bytes of a 16-B/lane coalesced stream
(doubled below as that guide prescribes); WRITE_SIZE is exact for 16-B/lane stores; other
widths are uncalibrated -- the forward kernel stores 4-8 B per lane, so the write figure is
reported as measured.  The warmup launches are dropped (first dispatches of the process)."""
import csv
import glob
import json
import os
import sys

out = sys.argv[1]
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    files = glob.glob(os.path.join(out, c, "**", "*counter_collection.csv"), recursive=True)
    vals = []
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") == c:
                    vals.append((int(row.get("Dispatch_Id", 0)), float(row["Counter_Value"]), row.get("Kernel_Name", "")))
    vals.sort()
    res[c] = vals
n = min(len(res["FETCH_SIZE"]), len(res["WRITE_SIZE"]))
half = n // 2  # bench: warmup 1 + steps 1 with the same number of launches each -> keep the timed half
fetch_kb = [v for _, v, _ in res["FETCH_SIZE"][half:]]
write_kb = [v for _, v, _ in res["WRITE_SIZE"][half:]]
fetch = 2.0 * 1024 * sum(fetch_kb) / max(len(fetch_kb), 1)
write = 1024 * sum(write_kb) / max(len(write_kb), 1)
print(json.dumps({
    "kernel": res["FETCH_SIZE"][0][2] if res["FETCH_SIZE"] else None,
    "launches_measured": len(fetch_kb),
    "fetch_bytes_per_launch_corrected_x2": fetch,
    "write_bytes_per_launch": write,
    "hbm_bytes_per_launch": fetch + write,
    "raw_fetch_kb": fetch_kb, "raw_write_kb": write_kb,
}, indent=1))
