#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_bw_tiny
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/debug/bw_tiny_diag.py 2>&1 | tee $O/diag.txt
