#!/bin/bash
# Round 5 session 11 (after the container re-creation): the full GPU suite at HEAD, smoke, the
# default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_s11
mkdir -p $O
cd $R
step() {
  local name=$1 t=$2
  shift 2
  echo "== $name" ; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  tail -3 $O/$name.log | cut -c1-400; echo "== $name rc=$rc"; return $rc
}
step pytest 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests &&
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
step bench 400 python -u bench.py &&
step c5_configs 300 python -u tools/bench_configs.py c5 &&
step c5_trace 300 env CV_TRACE=1 REPS=3 python -u tools/bench_configs.py c5
