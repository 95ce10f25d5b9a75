#!/bin/bash
# Round 5 session 8: f32 VALU microbench (bank conflicts, DPP) and the PMC basis regenerated
# from HEAD's kernels (f64 forward: roofline.traffic + clock; f32 pair trellis with the clock).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_s8
mkdir -p $O
cd $R
timeout -k 10 120 tools/microbench/f32_mix_rates > $O/f32mix.txt 2>&1 || exit 1
cat $O/f32mix.txt
TAG=r05_pmc_f64 T_PMC=200 bash tools/pmc_f64.sh > $O/pmc_f64.log 2>&1 || { tail -5 $O/pmc_f64.log; exit 1; }
tail -3 $O/pmc_f64.log
TAG=r05_pmc_f32 KRE=trellis_fwd2_f32 PMC_ARGS="--dtype f32" T_PMC=200 bash tools/pmc_f64.sh > $O/pmc_f32.log 2>&1 || { tail -5 $O/pmc_f32.log; exit 1; }
tail -3 $O/pmc_f32.log
