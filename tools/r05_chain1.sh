#!/bin/bash
# Round 5: the parallel CPSolver chain above N = 256 -- its GPU tests, then the 4,096 x 512
# parallel-vs-serial comparisons at N = 512 and 1,024 (tools/bench_chain_large_n.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_chain1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_chain_par.py \
  -k "large_n or serial_large" > $O/tests_chain.log 2>&1; rc=$?; tail -30 $O/tests_chain.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_large_n.py \
  -k "explicit_request or equal_batch_chunks" > $O/tests_large.log 2>&1; rc=$?; tail -8 $O/tests_large.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python -u tools/bench_chain_large_n.py 512 4096 > $O/bench_512.log 2>&1; rc=$?; cat $O/bench_512.log; [ $rc -eq 0 ] &&
timeout -k 10 400 python -u tools/bench_chain_large_n.py 1024 4096 > $O/bench_1024.log 2>&1; rc=$?; cat $O/bench_1024.log; exit $rc
