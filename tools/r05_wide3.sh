#!/bin/bash
# The pipelined wide kernel: its tests, the crossover at small / large N, the chain's speculation.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r05_wide3}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_large_n.py tests/test_gpu_chain_par.py -x -q --timeout 300 --timeout-method thread -m gpu -k "wide or beyond" > $OUT/pytest.log 2>&1 || { echo "pytest FAIL"; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python -u tools/bench_wide.py --n 256 --nseq 620 --T 512 --wide-s auto --assocs cp --chain-len 8 > $OUT/b256.log 2>&1 || { echo "b256 FAIL"; tail -5 $OUT/b256.log; exit 1; }
grep -v amdgpu $OUT/b256.log
timeout -k 10 400 python -u tools/bench_wide.py --n 1100,4096,10240 --nseq 4,64,1024 --T 8 --wide-s auto,1,4 --assocs viterbi --chain-len 64 > $OUT/bx.log 2>&1 || { echo "bx FAIL"; tail -5 $OUT/bx.log; exit 1; }
grep -v amdgpu $OUT/bx.log
