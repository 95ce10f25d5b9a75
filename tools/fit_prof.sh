#!/bin/bash
# fit kernels: tests, then a kernel trace of a config-4-shaped EM call per CV_BW_MT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R && timeout -k 10 300 python -u -m pytest tests/test_fit.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for mt in 2 4; do
  CV_BW_MT=$mt SHAPE=c4 ITERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mt$mt -o kt -- python3 $R/tools/bench_fit.py > $O/mt$mt.log 2>&1 || exit 1
done
