#!/bin/bash
# Baum-Welch E-step kernels under rocprofv3 --kernel-trace --stats at a quarter of config 4
# (16,384 x 512, N = 256): the in-tree library and each tools/_ab/lib_<v>.so of VARIANTS
# (default: the timing-only ablations nobnum norows noalpha, tools/build_fit_variant.sh).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r06_bwab
for v in base ${VARIANTS:-nobnum norows noalpha}; do
  if [ $v = base ]; then unset CV_LIB_PATH; else export CV_LIB_PATH=$R/tools/_ab/lib_$v.so; fi
  SHAPE=c4 BATCH=16384 ITERS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/gpurun_out/r06_bwab/$v -o s -- python3 $R/tools/bench_fit.py train > $R/gpurun_out/r06_bwab/$v.log 2>&1 || exit 1
  python3 - $R/gpurun_out/r06_bwab/$v/s_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "bw_" in n and ("mm" in n or "gemm" in n):
        print(sys.argv[2], n.split("(")[0][-30:], r["Calls"], f"{float(r['AverageNs']) / 1e6:.3f} ms")
PY
done
