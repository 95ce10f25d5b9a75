#!/bin/bash
# Round 5 session 9: software-pipelined f32 pair trellis (lib_pipe = -DCVK_F32_PIPE) -- f32
# parity tests on it, then interleaved A/B vs the in-tree build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_s9
mkdir -p $O
cd $R
CV_LIB_PATH=$R/tools/_ab/lib_pipe.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests_pipe.log 2>&1; rc=$?
tail -2 $O/tests_pipe.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="new pipe new pipe" bash tools/r05_session7.sh
