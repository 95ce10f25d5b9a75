#!/bin/bash
# generic_fwd_split with 512-thread workgroups (K = 512 / 64 ceil(N / 64)) and 16 candidate loads
# in flight: its tests, then the config-4-sized chain's speculative kernel per K (kernel trace).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r05_split2}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_large_n.py -k "split" -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest FAIL"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
for v in "1:2" "1:4" "0:"; do
  s=${v%%:*}; k=${v#*:}
  CV_GENERIC_SPLIT=$s CV_GENERIC_SPLIT_K=$k SERIAL=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$s$k -o kt -- python3 $R/tools/bench_chain_large_n.py 256 256 65536 > $OUT/run$s$k.log 2>&1 || { tail -5 $OUT/run$s$k.log; exit 1; }
  echo "split=$s K=$k: $(grep 'config-4-sized' $OUT/run$s$k.log | tail -1 | cut -c80-140) | $(grep -h 'generic_fwd' $OUT/kt$s$k/kt_kernel_stats.csv | cut -d, -f1-4 | tr '\n' ' ')" | tee -a $OUT/summary.txt
done
