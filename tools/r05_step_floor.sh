#!/bin/bash
# the per-step floor microbench (tools/microbench/step_floor.hip) at 620 and 2,480 sequences
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_step_floor
mkdir -p $O
for n in 620 2480 64; do
  timeout -k 10 120 $R/tools/microbench/step_floor $n | tee -a $O/out.txt || exit 1
done
