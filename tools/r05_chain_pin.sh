#!/bin/bash
# The chain's pinned chunked path copy: chain tests, then config-4-sized solves with the pinned
# chunks (default) vs the runtime's pageable copy (CV_CHAIN_PIN_COPY=0), interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_chain_pin
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain_par.py -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest FAIL"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for v in 1 0; do
    CV_CHAIN_PIN_COPY=$v SERIAL=0 timeout -k 10 200 python -u tools/bench_chain_large_n.py 256 256 65536 > $OUT/pin$v.$r.log 2>&1 || { echo "FAIL $v"; tail -5 $OUT/pin$v.$r.log; exit 1; }
    echo "pin=$v round $r: $(grep 'config-4-sized' $OUT/pin$v.$r.log | tail -1 | cut -c1-120)" | tee -a $OUT/summary.txt
  done
done
