#!/bin/bash
# HIP runtime API + kernel + copy trace of a config-4-sized parallel chain solve: which calls
# the device copies between the certificate pass and the quantised folds belong to.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_chain_api
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
SERIAL=0 timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv -d $OUT/t -o t -- python3 $R/tools/bench_chain_large_n.py 256 256 65536 > $OUT/run.log 2>&1 || { tail -5 $OUT/run.log; exit 1; }
python3 - $OUT/t <<'PY' | tee $OUT/timeline.txt
import csv, glob, os, sys
rows = []
def add(pattern, kind, name_key):
    for f in glob.glob(os.path.join(sys.argv[1], "**", pattern), recursive=True):
        for r in csv.DictReader(open(f)):
            nm = r.get(name_key, "") or ""
            if kind == "copy":
                nm = f"{r.get('Direction', '')} {r.get('Size', '')}"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, nm[:70]))
add("*kernel_trace.csv", "kern", "Kernel_Name")
add("*memory_copy_trace.csv", "copy", "Direction")
add("*hip_api_trace.csv", "api", "Function")
rows.sort()
i0 = max(i for i, r in enumerate(rows) if r[2] == "kern" and "cp_cert_f64" in r[3])
t0 = rows[i0][0]
for s, e, k, n in rows[i0 - 3:]:
    if k == "api" and n.startswith(("hipGetLastError", "hipPeekAtLastError", "hipGetDevice", "hipSetDevice")):
        continue
    print(f"{(s - t0) / 1e6:9.3f} -> {(e - t0) / 1e6:9.3f} ({(e - s) / 1e6:7.3f}) {k:4s} {n}")
PY
