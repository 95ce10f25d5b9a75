#!/bin/bash
# Round 5 final HEAD: the rocprofv3 kernel-trace summary of the bench and the two PMC traffic
# passes of the f64 forward (the same steps as tools/r05_final.sh after its bench).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_final4
mkdir -p $O
step() {
  local name=$1 t=$2
  shift 2
  echo "== $name" ; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  tail -3 $O/$name.log | cut -c1-300; echo "== $name rc=$rc"; return $rc
}
cd /tmp && export TMPDIR=/tmp &&
step prof 400 rocprofv3 --kernel-trace --stats -d $O/prof -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-f32-extra --no-configs &&
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-include-regex trellis_fwd_f64 -d $O/pmc1 -o p --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-f32-extra --no-configs &&
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex trellis_fwd_f64 -d $O/pmc2 -o p --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-f32-extra --no-configs
