#!/bin/bash
# The chain's speculative batch with S sequences per workgroup sharing each A load
# (CV_GENERIC_S=1/2/4, generic_fwd_ms) vs the candidate split: chain tests, then config-4-sized
# solves under a kernel trace per variant.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r05_spec_s}
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_chain_par.py tests/test_gpu_large_n.py -k "chain or multi_sequence or split" -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest FAIL"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-"0:2" "0:1" "0:4"}; do
  sp=${v%%:*}; s=${v#*:}
  CV_GENERIC_SPLIT=$sp CV_GENERIC_S=$s SERIAL=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$sp$s -o kt -- python3 $R/tools/bench_chain_large_n.py 256 256 65536 > $OUT/run$sp$s.log 2>&1 || { tail -5 $OUT/run$sp$s.log; exit 1; }
  python3 - $OUT/kt$sp$s/kt_kernel_stats.csv "split=$sp S=$s" <<'PY' | tee -a $OUT/summary.txt
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "generic_fwd" in r["Name"] or "trellis_fwd_f64<4" in r["Name"]:
        print(f"{sys.argv[2]}: {r['Name'].split('(')[0][-60:]} {float(r['AverageNs']) / 1e6:.2f} ms x{r['Calls']}")
PY
  grep 'config-4-sized' $OUT/run$sp$s.log | cut -c1-110 | tee -a $OUT/summary.txt
done
