#!/bin/bash
# A/B of bit-identical env knobs at several batches (the per-GPU shards of strong scaling and
# the full batch), interleaved on ONE box, after the f64 GPU tests (unless NO_TESTS):
#   AB="CV_X=0 CV_X=1" BATCHES="8192 65536" tools/ab_env_small.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-abenv}
mkdir -p $OUT
cd $R
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 ${T_TEST:-300} python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_constrained.py tests/test_gpu_fullsize.py -x -q \
    --timeout 200 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -20 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for B in ${BATCHES:-8192 16384}; do
    for v in $AB; do
      env $v timeout -k 10 ${T_BENCH:-200} python bench.py --batch $B --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-f32-extra --no-configs > $OUT/$v.$B.$r.log 2>&1 || { echo "FAIL $v $B"; tail -5 $OUT/$v.$B.$r.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], sys.argv[4], round(d['ms_per_step'],3), 'fwd', round(d['kernel_ms_per_step']['forward'],3), 'bt', round(d['kernel_ms_per_step']['backtrack_rescore'],3))" $OUT/$v.$B.$r.log $B $v $r | tee -a $OUT/summary.txt
    done
  done
done
