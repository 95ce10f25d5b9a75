#!/bin/bash
# the generic-kernel and chain GPU tests after a generic_fwd_ms change
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_generic_tests
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_n.py tests/test_gpu_chain_par.py tests/test_gpu_f64.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; exit $rc
