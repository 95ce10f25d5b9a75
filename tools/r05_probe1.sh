#!/bin/bash
# Round 5, first GPU session: the f64-MFMA co-issue microbench and the
# f32 trellis's kernel trace + SQ counters.  Each GPU step under its own
# time limit, chained with &&.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_probe1
mkdir -p $O
cd $R/tools/microbench && hipcc --offload-arch=gfx950 -O3 -o mfma_f64_coissue mfma_f64_coissue.hip &&
timeout -k 10 120 ./mfma_f64_coissue > $O/mfma_f64_coissue.txt 2>&1 && cat $O/mfma_f64_coissue.txt &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/f32trace -o p --output-format csv -- \
  python3 $R/bench.py --dtype f32 --steps 5 --warmup 2 --no-f32-extra --no-configs --no-cpu-baseline \
  > $O/f32trace.log 2>&1 && tail -3 $O/f32trace.log &&
KREGEX=trellis_fwd2_f32 BENCH_ARGS="--dtype f32 --no-f32-extra --no-configs" T_PMC=200 bash $R/tools/pmc_sq.sh \
  > $O/f32_sq.txt 2>&1 && cp -r $R/gpurun_out/pmc_sq $O/f32_sq && cat $O/f32_sq.txt
