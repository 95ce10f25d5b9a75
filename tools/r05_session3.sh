#!/bin/bash
# Round 5 session 3: f32 VALU mix microbench; S per wave for the NP = 512 / 1,024 units
# (large-N decode throughput, the parallel chain at N = 512 / 1,024), their GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_s3
mkdir -p $O
cd $R
step() {
  local name=$1 t=$2
  shift 2
  echo "== $name" ; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  tail -12 $O/$name.log; echo "== $name rc=$rc"; return $rc
}
step f32mix 120 tools/microbench/f32_mix_rates &&
step large_n_4096 300 env NSEQ=4096 python -u tools/bench_large_n.py 512 800 1024 &&
step large_n_16384 300 env NSEQ=16384 python -u tools/bench_large_n.py 512 1024 &&
step chain_1024 300 env SERIAL=0 python -u tools/bench_chain_large_n.py 1024 4096 &&
step chain_512 300 env SERIAL=0 python -u tools/bench_chain_large_n.py 512 4096 &&
step tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_large_n.py tests/test_gpu_chain_par.py
