#!/bin/bash
# SQ counters of the forward kernels in the ablation harness (tools/microbench/fwd_ablate),
# one --pmc pass per counter group and kernel kind (0 = 1 seq/WG, 1 = 2 seq/WG).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_ablate
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for K in ${KINDS:-0 1}; do
  i=0
  for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU"; do
    i=$((i + 1))
    timeout -k 10 120 rocprofv3 --pmc $G -d $OUT/k$K/g$i -o p --output-format csv -- \
      $R/tools/microbench/fwd_ablate_base 8192 $K > $OUT/k$K.g$i.log 2>&1 || exit $?
  done
done
python3 - "$OUT" <<'PY' > $OUT/summary.txt
import csv, glob, os, sys, collections
out = sys.argv[1]
for kd in sorted(glob.glob(os.path.join(out, "k*"))):
    if not os.path.isdir(kd):
        continue
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(kd, "g*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
            disp[row["Counter_Name"]].add(row.get("Dispatch_Id", "0"))
    print(f"== {os.path.basename(kd)} (per dispatch)")
    for k in sorted(tot):
        print(f"  {k:28s} {tot[k] / max(len(disp[k]), 1):.4e}")
    w = tot.get("SQ_WAVE_CYCLES", 0)
    for k in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
              "SQ_ACTIVE_INST_ANY"):
        if w and k in tot:
            print(f"  {k} / SQ_WAVE_CYCLES = {tot[k] / w:.3f}")
PY
cat $OUT/summary.txt
