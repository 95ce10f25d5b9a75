#!/bin/bash
# SQ counters of every trellis_fwd_f64 dispatch of one config-5 decode without the side stream
# (prefix pass, suffix pass, resume forward), one --pmc pass per group.  Usage: tools/pmc_c5_ext.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_c5_ext}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_WAVES" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD"; do
  i=$((i + 1))
  CV_NO_SIDE=1 REPS=1 timeout -k 10 -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex "trellis_fwd_f64" -d $OUT/g$i -o p \
    --output-format csv -- python3 $R/tools/bench_configs.py c5 > $OUT/g$i.log 2>&1 || exit $?
done
python3 - "$OUT" <<'PY' > $OUT/summary.txt
import csv, glob, os, sys, collections
out = sys.argv[1]
rows = collections.defaultdict(dict)
for f in glob.glob(os.path.join(out, "g*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        rows[(int(r["Dispatch_Id"]), r["Kernel_Name"][:90])][r["Counter_Name"]] = rows[(int(r["Dispatch_Id"]), r["Kernel_Name"][:90])].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for (d, k), c in sorted(rows.items()):
    w = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(d, k)
    print("   " + "  ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
    print(f"   VALU/wave-cycles={c.get('SQ_ACTIVE_INST_VALU', 0) / w:.3f} WAIT_ANY={c.get('SQ_WAIT_ANY', 0) / w:.3f}"
          f" WAIT_INST_ANY={c.get('SQ_WAIT_INST_ANY', 0) / w:.3f} GUI_ms={c.get('GRBM_GUI_ACTIVE', 0) / 8 / 2.25e6:.2f}")
PY
cat $OUT/summary.txt
