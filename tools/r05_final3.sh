#!/bin/bash
# Round 5's last GPU session: the chain's u8 path copy A/B (config-4-sized solves, interleaved),
# then the full GPU suite, smoke and the default bench line at HEAD.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_final3
mkdir -p $O
cd $R
step() {
  local name=$1 t=$2
  shift 2
  echo "== $name" ; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  tail -3 $O/$name.log | cut -c1-300; echo "== $name rc=$rc"; return $rc
}
step chain_tests 400 python -u -m pytest tests/test_gpu_chain_par.py -x -q --timeout 200 --timeout-method thread -m gpu || exit 1
for r in 1 2; do
  for v in 1 0; do
    CV_CHAIN_U8=$v SERIAL=0 timeout -k 10 200 python -u tools/bench_chain_large_n.py 256 256 65536 > $O/u8_$v.$r.log 2>&1 || { echo "FAIL u8 $v"; exit 1; }
    echo "u8=$v round $r: $(grep 'config-4-sized' $O/u8_$v.$r.log | tail -1 | cut -c1-120)" | tee -a $O/summary.txt
  done
done
step pytest 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests &&
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
step bench 400 python -u bench.py
