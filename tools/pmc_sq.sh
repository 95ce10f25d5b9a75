#!/bin/bash
# SQ issue/stall counters of the forward trellis kernel (one --pmc pass per group, kernel
# trace only).  Usage: tools/pmc_sq.sh  (env BENCH_ARGS passes bench.py options).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_sq
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
         "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU"; do
  i=$((i + 1))
  timeout -k 10 ${T_PMC:-300} rocprofv3 --pmc $G --kernel-include-regex "${KREGEX:-trellis_fwd}" -d $OUT/g$i -o p \
    --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} \
    > $OUT/g$i.log 2>&1 || exit $?
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
    print(f"{k:28s} {tot[k]:.4e}  (rows {n[k]})")
w = tot.get("SQ_WAVE_CYCLES", 0)
if w:
    for k in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
              "SQ_ACTIVE_INST_ANY"):
        if k in tot:
            print(f"{k} / SQ_WAVE_CYCLES = {tot[k] / w:.3f}")
PY
cat $OUT/summary.txt
