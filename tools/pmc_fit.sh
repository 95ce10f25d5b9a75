#!/bin/bash
# SQ counters of the Baum-Welch E-step kernels (64 < N <= 256) on a config-4-shaped corpus,
# one --pmc pass per group, kernel trace only.  Usage: tools/pmc_fit.sh TAG [kernel regex]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_fit}
KRE=${2:-bw_}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM"; do
  i=$((i + 1))
  SHAPE=c4 ITERS=1 timeout -k 10 -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex "$KRE" -d $OUT/g$i -o p \
    --output-format csv -- python3 $R/tools/bench_fit.py > $OUT/g$i.log 2>&1 || exit $?
done
python3 - "$OUT" <<'PY' > $OUT/summary.txt
import csv, glob, os, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(os.path.join(out, "g*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "")
        tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
for k, d in sorted(tot.items()):
    print(k)
    for c in sorted(d):
        print(f"  {c:28s} {d[c]:.4e}")
    w = d.get("SQ_WAVE_CYCLES", 0)
    for c in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
        if w and c in d:
            print(f"  {c} / SQ_WAVE_CYCLES = {d[c] / w:.3f}")
    if d.get("GRBM_GUI_ACTIVE") and d.get("SQ_VALU_MFMA_BUSY_CYCLES"):
        print(f"  MFMA busy per SIMD-cycle = {d['SQ_VALU_MFMA_BUSY_CYCLES'] / (d['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}"
              " (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 XCDs x 1024 SIMDs))")
PY
cat $OUT/summary.txt
