#!/bin/bash
# Quick GPU session: a pytest selection (PYSEL), the default bench, a rocprofv3 kernel-trace
# summary of the bench.  Each GPU step has its own time limit and the steps stop at the first
# failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${TAG:-quick}
if [ -n "${PYSEL:-}${PYK:-}" ]; then
  timeout -k 10 ${T_TEST:-600} python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu ${PYSEL:-} \
    ${PYK:+-k "$PYK"} \
    > $OUT/${TAG}_pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -4 $OUT/${TAG}_pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "${NO_BENCH:-}" ]; then
  timeout -k 10 ${T_BENCH:-400} python -u bench.py ${BENCH_ARGS:---steps 10 --warmup 2} > $OUT/${TAG}_bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -c 3000 $OUT/${TAG}_bench.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "${NO_PROF:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 ${T_PROF:-400} rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o kt --output-format csv -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs > $OUT/${TAG}_prof.log 2>&1; rc=$?
  echo "rocprof rc=$rc"
  f=$(find $OUT/${TAG}_prof -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cut -d, -f1-8 "$f" | head -12
  exit $rc
fi
