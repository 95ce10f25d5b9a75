#!/bin/bash
# HBM traffic of the forward trellis kernel: two separate --pmc passes (FETCH_SIZE and
# WRITE_SIZE do not fit one pass on gfx950), kernel-trace only, no sys/runtime trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${T_PMC:-300} rocprofv3 --pmc $C --kernel-include-regex "trellis_(fwd|mfma)" -d $OUT/$C -o p \
    --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} \
    > $OUT/$C.log 2>&1 || exit $?
done
python3 $R/tools/pmc_summary.py $OUT > $OUT/summary.json && cat $OUT/summary.json
