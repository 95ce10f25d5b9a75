#!/bin/bash
# Round 5 end-of-round measurement at HEAD: the full GPU suite, smoke, the default bench line,
# a rocprofv3 kernel-trace summary of the bench (its forward's average must agree with the
# line's HIP-event kernel time), and one PMC traffic pass of the f64 forward.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r05_final}
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
step bench 400 python -u bench.py &&
cd /tmp && export TMPDIR=/tmp &&
step prof 400 rocprofv3 --kernel-trace --stats -d $O/prof -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-f32-extra --no-configs &&
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-include-regex trellis_fwd_f64 -d $O/pmc1 -o p --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-f32-extra --no-configs &&
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex trellis_fwd_f64 -d $O/pmc2 -o p --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-f32-extra --no-configs
