#!/bin/bash
# Small-batch A/B (the per-GPU shards of 8-GPU / 4-GPU strong scaling): f64 GPU tests on the
# NEW library, then VARIANTS interleaved at BATCHES.  Usage: VARIANTS="old db" tools/ab_small.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-absmall}
mkdir -p $OUT
cd $R
LIB=consistent-viterbi_amd/cviterbi/libcviterbi.so
NEW=${NEW:-$(echo ${VARIANTS:-old new} | awk '{print $NF}')}
export CV_LIB_PATH=$(pwd)/tools/_ab/lib_$NEW.so
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 ${T_TEST:-300} python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_constrained.py tests/test_gpu_fullsize.py -x -q \
    --timeout 200 --timeout-method thread -m gpu > $OUT/pytest_$NEW.log 2>&1 || { echo "pytest failed"; tail -20 $OUT/pytest_$NEW.log; exit 1; }
  tail -1 $OUT/pytest_$NEW.log
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for B in ${BATCHES:-8192 16384}; do
    for v in ${VARIANTS:-old new}; do
      export CV_LIB_PATH=$(pwd)/tools/_ab/lib_$v.so
      timeout -k 10 ${T_BENCH:-200} python bench.py --batch $B --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-f32-extra > $OUT/$v.$B.$r.log 2>&1 || { echo "FAIL $v $B"; tail -5 $OUT/$v.$B.$r.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], sys.argv[4], round(d['ms_per_step'],3), 'fwd', round(d['kernel_ms_per_step']['forward'],3), 'bt', round(d['kernel_ms_per_step']['backtrack_rescore'],3))" $OUT/$v.$B.$r.log $B $v $r | tee -a $OUT/summary.txt
    done
  done
done
export CV_LIB_PATH=$(pwd)/tools/_ab/lib_$NEW.so
