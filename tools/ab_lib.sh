#!/bin/bash
# A/B of two builds of libcviterbi.so (tools/_ab/lib_<variant>.so built in this container, VARIANTS="old new ...") on
# the config-4 bench, interleaved on ONE box: ROUNDS=2 BENCH_ARGS=... tools/ab_lib.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-ablib}
mkdir -p $OUT
cd $R
LIB=consistent-viterbi_amd/cviterbi/libcviterbi.so
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-old new}; do
    export CV_LIB_PATH=$(pwd)/tools/_ab/lib_$v.so
    timeout -k 10 ${T_BENCH:-240} python bench.py ${BENCH_ARGS:---steps 8 --warmup 2 --no-cpu-baseline --no-f32-extra} > $OUT/$v.$r.log 2>&1 || { echo "FAIL $v"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],2), 'fwd', round(d['kernel_ms_per_step']['forward'],2), 'bt', round(d['kernel_ms_per_step']['backtrack_rescore'],2))" $OUT/$v.$r.log $v $r | tee -a $OUT/summary.txt
  done
done
