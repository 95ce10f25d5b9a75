#!/bin/bash
# Wide decode after the XCD-mapping fix: tests, N = 256 x 620 (cp), the small-batch crossover,
# N = 10,240 with the XCD-aware mapping on / off; the chain tests with the default speculation.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r05_wide4}
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_large_n.py tests/test_gpu_chain_par.py -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest FAIL"; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python -u tools/bench_wide.py --n 256 --nseq 620 --T 512 --wide-s auto --assocs cp --chain-len 8 > $OUT/b256.log 2>&1 || { echo "b256 FAIL"; tail -5 $OUT/b256.log; exit 1; }
grep -v amdgpu $OUT/b256.log
timeout -k 10 300 python -u tools/bench_wide.py --n 1100,2048,4096 --nseq 4,64,1024 --T 8 --wide-s auto,1,4 --assocs viterbi --chain-len 64 > $OUT/bx.log 2>&1 || { echo "bx FAIL"; tail -5 $OUT/bx.log; exit 1; }
grep -v amdgpu $OUT/bx.log
for x in 1 0; do
  CV_WIDE_XCD=$x timeout -k 10 300 python -u tools/bench_wide.py --n 10240 --nseq 4,64,1024 --T 8 --wide-s auto --assocs viterbi --chain-len 64 > $OUT/b10k_xcd$x.log 2>&1 || { echo "b10k FAIL"; tail -5 $OUT/b10k_xcd$x.log; exit 1; }
  echo "== CV_WIDE_XCD=$x"; grep -v amdgpu $OUT/b10k_xcd$x.log
done
