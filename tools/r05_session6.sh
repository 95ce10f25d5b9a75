#!/bin/bash
# Round 5 session 6: generic kernels' unrolled candidate loops + one-state-per-thread single-
# sequence workgroups: tests, then A/B (lib_roll = CVK_GEN_UNROLL=1) on the large-N decode and
# the parallel chain's speculation above N = 256; f32 CV_F32_ONEBAR re-A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_s6
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_large_n.py tests/test_gpu_chain_par.py tests/test_gpu_configs_oracle.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in roll new; do
    CV_LIB_PATH=$R/tools/_ab/lib_$v.so NSEQ=4096 timeout -k 10 300 python -u tools/bench_large_n.py 300 600 > $O/large_$v.$r.log 2>&1 || exit 1
    sed "s/^/$v $r /" $O/large_$v.$r.log | grep "N=" | tee -a $O/summary.txt
    CV_LIB_PATH=$R/tools/_ab/lib_$v.so CV_TRACE=1 SERIAL=0 timeout -k 10 300 python -u tools/bench_chain_large_n.py 1024 4096 > $O/chain1024_$v.$r.log 2>&1 || exit 1
    grep "walk\|parallel\|again" $O/chain1024_$v.$r.log | sed "s/^/$v $r /" | tail -4 | tee -a $O/summary.txt
  done
done
for r in 1 2 3; do
  for ob in 0 1; do
    CV_F32_ONEBAR=$ob timeout -k 10 240 python bench.py --dtype f32 --steps 8 --warmup 2 --no-cpu-baseline --no-f32-extra \
      --no-configs > $O/f32_$ob.$r.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('onebar', sys.argv[2], sys.argv[3], round(d['ms_per_step'],2), 'fwd', round(d['kernel_ms_per_step']['forward'],2))" $O/f32_$ob.$r.log $ob $r | tee -a $O/summary.txt
  done
done
