#!/bin/bash
# Round 5, at the HEAD after reverting the neutral chain copy experiments (u8 paths, prefault):
# the full GPU suite, smoke, the bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_final4
mkdir -p $O
cd $R
step() {
  local name=$1 t=$2
  shift 2
  echo "== $name" ; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  tail -3 $O/$name.log | cut -c1-300; echo "== $name rc=$rc"; return $rc
}
step pytest 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests &&
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
step bench 400 python -u bench.py
