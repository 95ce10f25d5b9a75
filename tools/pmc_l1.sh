#!/bin/bash
# L1 / L2 hit counters of the f64 forward (trellis_fwd_f64) for library variants
# (tools/_ab/lib_<v>.so), one --pmc pass each, NSEQ sequences of config 4 (tools/t64_sweep.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-pmc_l1}
mkdir -p $OUT
LIB=$R/consistent-viterbi_amd/cviterbi/libcviterbi.so
cd /tmp && export TMPDIR=/tmp
export NSEQ=${NSEQ:-16384}
for v in ${VARIANTS:-base}; do
  export CV_LIB_PATH=$R/tools/_ab/lib_$v.so
  timeout -s KILL 120 rocprofv3 --pmc ${COUNTERS:-TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum} \
    --kernel-include-regex "trellis_fwd_f64" -d $OUT/$v -o p --output-format csv -- python3 $R/tools/t64_sweep.py \
    > $OUT/$v.log 2>&1 || exit 1
done
python3 - "$OUT" ${VARIANTS:-base} <<'PY' | tee $OUT/summary.txt
import csv, glob, os, sys, collections
out = sys.argv[1]
for v in sys.argv[2:]:
    tot = collections.defaultdict(float)
    for f in glob.glob(os.path.join(out, v, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
    s = " ".join(f"{k}={tot[k]:.4e}" for k in sorted(tot))
    r = tot["TCP_TCC_READ_REQ_sum"] / max(tot["TCP_TOTAL_CACHE_ACCESSES_sum"], 1)
    h = tot["TCC_HIT_sum"] / max(tot["TCC_HIT_sum"] + tot["TCC_MISS_sum"], 1)
    print(f"{v}: L1->L2 reads / L1 accesses {r:.3f}  L2 hit {h:.3f}  {s}")
PY
