#!/bin/bash
# Round 5 session 4: one barrier per step in the f32 pair trellis (CV_F32_ONEBAR): parity tests
# with the knob on, then the config-4 f32 A/B interleaved on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_s4
mkdir -p $O
cd $R
CV_F32_ONEBAR=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_constrained.py > $O/tests_onebar.log 2>&1; rc=$?
tail -3 $O/tests_onebar.log; [ $rc -eq 0 ] &&
TAG=r05_s4/ab AB="CV_F32_ONEBAR=0 CV_F32_ONEBAR=1" ROUNDS=3 \
  BENCH_ARGS="--dtype f32 --steps 8 --warmup 2 --no-cpu-baseline --no-f32-extra --no-configs" bash tools/ab_env.sh
