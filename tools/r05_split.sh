#!/bin/bash
# generic_fwd_split (K threads per state, the small-batch psi-mode default below N = 512): its
# tests and the generic / chain suites, then config-4-sized gpu-cp solves with the speculative
# batch on the split kernel (CV_GENERIC_SPLIT=1) vs one thread per state (=0), interleaved, and
# one traced solve each (the speculative batch's phase).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r05_split}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_n.py tests/test_gpu_chain_par.py -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest FAIL"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for v in 1 0; do
    CV_GENERIC_SPLIT=$v SERIAL=0 timeout -k 10 200 python -u tools/bench_chain_large_n.py 256 256 65536 > $OUT/sp$v.$r.log 2>&1 || { echo "FAIL $v"; tail -5 $OUT/sp$v.$r.log; exit 1; }
    echo "split=$v round $r: $(grep 'config-4-sized' $OUT/sp$v.$r.log | tail -1 | cut -c1-120)" | tee -a $OUT/summary.txt
  done
done
for v in 1 0; do
  CV_TRACE=1 CV_GENERIC_SPLIT=$v SERIAL=0 timeout -k 10 200 python -u tools/bench_chain_large_n.py 256 256 65536 > $OUT/trace$v.log 2>&1 || { echo "FAIL trace $v"; exit 1; }
  echo "split=$v traced: $(grep 'speculative' $OUT/trace$v.log | tail -2 | tr '\n' ' ')" | tee -a $OUT/summary.txt
done
