#!/bin/bash
# trellis_cp_f64 at one sequence per wave: the CP tests and the chain tests, then the
# config-4-sized chain's speculative batch on it (CV_CHAIN_SPEC_KERNEL=trellis, S = 1 and the
# old S = 2) vs generic_fwd_ms<1> (the default), kernel-traced.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_cp_s1
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_chain_par.py -k "cp or chain" -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest FAIL"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
for v in "trellis:1" "trellis:2" "generic:"; do
  k=${v%%:*}; s=${v#*:}
  CV_CHAIN_SPEC_KERNEL=$k CV_T64_CP_S=$s SERIAL=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$k$s -o kt -- python3 $R/tools/bench_chain_large_n.py 256 256 65536 > $OUT/run$k$s.log 2>&1 || { tail -5 $OUT/run$k$s.log; exit 1; }
  python3 - $OUT/kt$k$s/kt_kernel_stats.csv "spec=$k S=$s" <<'PY' | tee -a $OUT/summary.txt
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "generic_fwd" in r["Name"] or "trellis_cp_f64" in r["Name"] or "trellis_fwd_f64<4" in r["Name"]:
        print(f"{sys.argv[2]}: {r['Name'].split('(')[0][-50:]} {float(r['AverageNs']) / 1e6:.2f} ms x{r['Calls']}")
PY
  grep 'config-4-sized' $OUT/run$k$s.log | cut -c1-110 | tee -a $OUT/summary.txt
done
