#!/bin/bash
# A/B of libcviterbi.so builds (tools/_ab/lib_<v>.so) on the Baum-Welch E-step kernels at
# config-4 shape: kernel times from a rocprofv3 kernel trace, interleaved on ONE box.
# Usage: VARIANTS="a b a@CV_X=1,CV_Y=2" ROUNDS=2 TAG=... tools/ab_fit.sh (name@env: the build with env vars)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-abfit}
mkdir -p $OUT
LIB=$R/consistent-viterbi_amd/cviterbi/libcviterbi.so
for r in $(seq 1 ${ROUNDS:-2}); do
  for vv in ${VARIANTS:-a b}; do
    v=${vv%%@*}; ENVS=""; [ "$vv" != "$v" ] && ENVS=$(echo "${vv#*@}" | tr ',' ' ')
    export CV_LIB_PATH=$R/tools/_ab/lib_$v.so  # the variant, never copied over the in-tree .so
    (cd /tmp && env $ENVS TMPDIR=/tmp SHAPE=c4 ITERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $OUT/$vv.$r -o kt -- python3 $R/tools/bench_fit.py > $OUT/$vv.$r.log 2>&1) || { echo "FAIL $vv"; exit 1; }
    python3 - $OUT/$vv.$r/kt_kernel_stats.csv $vv $r <<'PY' | tee -a $OUT/summary.txt
import csv, sys
row = [f"{sys.argv[2]} {sys.argv[3]}"]
for r in csv.DictReader(open(sys.argv[1])):
    if "bw_" in r["Name"] and "mstep" not in r["Name"]:
        row.append(f'{r["Name"].split("(")[0].replace("void cvf::", "")} {float(r["AverageNs"]) / 1e6:.2f}')
print("  ".join(row))
PY
  done
done
