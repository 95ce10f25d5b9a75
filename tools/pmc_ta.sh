#!/bin/bash
# TA / TCP (vector L1) PMC passes over trellis_fwd_f64 for two library builds
# (tools/_ab/lib_<v>.so): is the vector memory path the limit once the delta stores are added?
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-pmc_ta}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for G in "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE" "TA_DATA_STALLED_BY_TC_CYCLES TA_BUFFER_WRITE_WAVEFRONTS" \
         "TCP_PENDING_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_RFIFO_STALL_CYCLES TCP_LFIFO_STALL_CYCLES"; do
  i=$((i + 1))
  for v in ${VARIANTS:-base NOSTORE}; do
    export CV_LIB_PATH=$R/tools/_ab/lib_$v.so
    NSEQ=65536 timeout -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex trellis_fwd_f64 -d $OUT/$v.g$i -o p \
      --output-format csv -- python3 $R/tools/bench_assoc.py viterbi > $OUT/$v.g$i.log 2>&1 || exit $?
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
res = collections.defaultdict(dict)
for d in sorted(glob.glob(os.path.join(out, "*.g*"))):
    if not os.path.isdir(d): continue
    v = os.path.basename(d).split(".")[0]
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            rows[r["Counter_Name"]].append((int(r.get("Dispatch_Id", 0)), float(r["Counter_Value"])))
        for k, x in rows.items():
            x.sort()
            res[v][k] = x[-1][1]  # last dispatch (the timed decode)
for v, c in res.items():
    print(v, {k: f"{x:.4e}" for k, x in sorted(c.items())})
    g = c.get("GRBM_GUI_ACTIVE")
    if g:
        cyc = g / 8
        for k in ("TA_TA_BUSY", "TA_ADDR_STALLED_BY_TC_CYCLES", "TA_DATA_STALLED_BY_TC_CYCLES", "TCP_PENDING_STALL_CYCLES",
                  "TCP_READ_TAGCONFLICT_STALL_CYCLES", "TCP_RFIFO_STALL_CYCLES", "TCP_LFIFO_STALL_CYCLES"):
            if k in c:
                print(f"  {k} per CU-cycle = {c[k] / 256 / cyc:.3f}")
PY
