#!/bin/bash
# Kernel trace of a config-4-sized parallel chain solve (N = 256): what the speculative batch's
# ~15 ms are made of.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r05_spec_trace}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
SERIAL=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/kt -o kt -- python3 $R/tools/bench_chain_large_n.py 256 256 65536 > $OUT/run.log 2>&1 || { tail -5 $OUT/run.log; exit 1; }
tail -2 $OUT/run.log
python3 - $OUT/kt <<'PY' | tee $OUT/timeline.txt
import csv, glob, os, sys
rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:90]))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", "") + " " + r.get("Size", "")))
rows.sort()
# the last solve: from the last trellis_fwd_f64 dispatch on
i0 = max(i for i, r in enumerate(rows) if "trellis_fwd_f64" in r[2])
t0 = rows[i0][0]
prev = None
for s, e, k in rows[i0:]:
    gap = "" if prev is None else f" (+{(s - prev) / 1e6:.3f} after prev end)"
    print(f"{(s - t0) / 1e6:9.3f} -> {(e - t0) / 1e6:9.3f} ms ({(e - s) / 1e6:8.3f}) {k}{gap}")
    prev = e
PY
