#!/bin/bash
# SQ issue/stall counters of any program's kernels (one --pmc pass per group, kernel trace
# only).  Usage: tools/pmc_prog.sh OUTDIR KERNEL_REGEX PROGRAM [ARGS...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
KRE=$2
shift 2
PROG=$(readlink -f "$1")
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
         "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU"; do
  i=$((i + 1))
  timeout -s KILL 60 rocprofv3 --pmc $G --kernel-include-regex "$KRE" -d $OUT/g$i -o p \
    --output-format csv -- $PROG "$@" > $OUT/g$i.log 2>&1 || exit $?
done
python3 - "$OUT" <<'PY' > $OUT/summary.txt
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float)
n = collections.defaultdict(int)
for f in glob.glob(out + "/g*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
for k in sorted(tot):
    print(f"{k:24s} {tot[k]:.4g}  (rows {n[k]})")
PY
cat $OUT/summary.txt
