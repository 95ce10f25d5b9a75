#!/bin/bash
# Round 5 session 5: f32 pair trellis waitcnt fixes -- parity tests of the in-tree build (both
# barrier layouts), then library variants x CV_F32_ONEBAR interleaved on one box (config 4 f32).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_s5
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
CV_F32_ONEBAR=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests_onebar.log 2>&1; rc=$?
tail -2 $O/tests_onebar.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for vv in r04@0 await@0 new@0 new@1; do
    v=${vv%@*}; ob=${vv#*@}
    CV_LIB_PATH=$R/tools/_ab/lib_$v.so CV_F32_ONEBAR=$ob timeout -k 10 240 python bench.py --dtype f32 --steps 8 --warmup 2 \
      --no-cpu-baseline --no-f32-extra --no-configs > $O/$vv.$r.log 2>&1 || { echo "FAIL $vv"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],2), 'fwd', round(d['kernel_ms_per_step']['forward'],2), 'bt', round(d['kernel_ms_per_step']['backtrack_rescore'],2))" $O/$vv.$r.log $vv $r | tee -a $O/summary.txt
  done
done
# where the parallel chain's time goes above N = 256 (host phase stamps)
CV_TRACE=1 SERIAL=0 timeout -k 10 300 python -u tools/bench_chain_large_n.py 1024 4096 > $O/chain_1024_trace.log 2>&1 || exit 1
grep -v amdgpu.ids $O/chain_1024_trace.log | tail -20
CV_TRACE=1 SERIAL=0 timeout -k 10 300 python -u tools/bench_chain_large_n.py 512 4096 > $O/chain_512_trace.log 2>&1 || exit 1
grep -v amdgpu.ids $O/chain_512_trace.log | tail -20
