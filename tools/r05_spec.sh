#!/bin/bash
# The parallel chain's speculative batch on trellis_cp_f64 vs generic_fwd_ms (CV_CHAIN_SPEC_KERNEL)
# at config-4 size (N = 256), traced; then the chain tests with the generic speculation.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r05_spec}
mkdir -p $OUT
cd $R
for k in trellis generic wide trellis generic wide; do
  W=""; [ $k = wide ] && W=1
  CV_GENERIC_WIDE_MIN=$W CV_TRACE=1 CV_CHAIN_SPEC_KERNEL=${k/wide/generic} SERIAL=0 timeout -k 10 200 python -u tools/bench_chain_large_n.py 256 256 65536 > $OUT/$k.log 2>&1 || { echo "FAIL $k"; tail -5 $OUT/$k.log; exit 1; }
  echo "== $k"; grep -E "speculative|walk|D2H|config-4-sized" $OUT/$k.log | tail -12
done
[ -n "$NO_TESTS" ] && exit 0
CV_CHAIN_SPEC_KERNEL=generic timeout -k 10 300 python -u -m pytest tests/test_gpu_chain_par.py -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest FAIL"; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
