#!/bin/bash
# One GPU session: parity tests, a short bench, a rocprofv3 kernel-trace profile.
# Each GPU step has its own time limit; steps are chained with && so a failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 ${T_TEST:-900} python -m pytest tests -x -q -m gpu ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 ${T_BENCH:-400} python bench.py ${BENCH_ARGS:---steps 5 --warmup 2} > $OUT/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -2 $OUT/bench.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${T_PROF:-400} rocprofv3 --kernel-trace --stats -T -d $OUT/prof -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -2 $OUT/prof.log
find $OUT/prof -name "*stats*" | head
exit $rc
