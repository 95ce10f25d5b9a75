#!/bin/bash
# PMC passes over the exact-f64 forward kernel (trellis_fwd_f64) on one config-4 chunk of
# 16,384 sequences (tools/t64_sweep.py).  One --pmc group per run, kernel trace only.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_t64
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export NSEQ=${NSEQ:-16384}
i=0
for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS" \
         "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum" \
         "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i + 1))
  timeout -k 10 ${T_PMC:-240} rocprofv3 --pmc $G --kernel-include-regex "trellis_fwd_f64" -d $OUT/g$i -o p \
    --output-format csv -- python3 $R/tools/t64_sweep.py > $OUT/g$i.log 2>&1 || exit $?
done
python3 - "$OUT" <<'PY' > $OUT/summary.txt
import csv, glob, os, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float)
n = collections.defaultdict(int)
for f in glob.glob(os.path.join(out, "g*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        tot[row["Counter_Name"]] += float(row["Counter_Value"])
        n[row["Counter_Name"]] += 1
for k in sorted(tot):
    print(f"{k:30s} {tot[k]:.4e}  (rows {n[k]})")
w = tot.get("SQ_WAVE_CYCLES", 0)
if w:
    for k in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
              "SQ_ACTIVE_INST_ANY"):
        if k in tot:
            print(f"{k} / SQ_WAVE_CYCLES = {tot[k] / w:.3f}")
if tot.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
    print(f"L1 -> L2 read requests / L1 accesses = {tot['TCP_TCC_READ_REQ_sum'] / tot['TCP_TOTAL_CACHE_ACCESSES_sum']:.3f}")
if tot.get("TCC_HIT_sum") is not None and tot.get("TCC_MISS_sum") is not None:
    print(f"L2 hit rate = {tot['TCC_HIT_sum'] / max(tot['TCC_HIT_sum'] + tot['TCC_MISS_sum'], 1):.3f}")
PY
cat $OUT/summary.txt
