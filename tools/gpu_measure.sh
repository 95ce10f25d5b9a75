#!/bin/bash
# Full measurement session at HEAD (one box): every GPU test, the default bench line, a
# rocprofv3 kernel-trace/stats profile of the same bench, PMC passes over the f64 forward and
# backtrack kernels, and the other configs.  Each GPU step has its own time limit and the
# session stops at the first failure.  Outputs under gpurun_out/$TAG/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-measure}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
step() { echo "[$(date +%T)] $*"; }
if [ -z "${NO_TESTS:-}" ]; then
  step pytest
  timeout -k 10 ${T_TEST:-900} python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu \
    > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -20 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
step bench
timeout -k 10 ${T_BENCH:-400} python -u bench.py ${BENCH_ARGS:---steps 10 --warmup 2} > $OUT/bench.log 2>&1 \
  || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -c 2500 $OUT/bench.log
step rocprof
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 ${T_PROF:-400} rocprofv3 --kernel-trace --stats -d $OUT/prof -o kt \
    --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-configs > $OUT/prof.log 2>&1 ) \
  || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -d, -f1-4 "$f" | head -8
if [ -z "${NO_PMC:-}" ]; then
  for K in trellis_fwd_f64 backtrack_f64; do
    step pmc $K
    TAG=$TAG/pmc_$K KRE=$K bash tools/pmc_f64.sh > $OUT/pmc_$K.txt 2>&1 || { echo "pmc $K failed"; tail $OUT/pmc_$K.txt; exit 1; }
    tail -12 $OUT/pmc_$K.txt
  done
fi
if [ -z "${NO_CONFIGS:-}" ]; then
  step configs
  timeout -k 10 ${T_CFG:-400} python -u tools/bench_configs.py ${CONFIGS:-c2 c2f64 c3 c3f64 c5 c5f32 c5host} > $OUT/configs.txt 2>&1 \
    || { echo "configs failed"; tail -20 $OUT/configs.txt; exit 1; }
  cat $OUT/configs.txt
fi
step done
