#!/bin/bash
# Baum-Welch E-step pipeline A/B (CV_BW_PIPE = parts per chunk on their own streams) at config-4
# shape: the fit tests, then per variant a kernel trace of tools/bench_fit.py and the EM iteration
# span (consecutive M-step ends within one call) -- interleaved on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r05_bwpipe}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fit.py > $O/pytest_fit.log 2>&1 || { tail -20 $O/pytest_fit.log; exit 1; }
tail -2 $O/pytest_fit.log
cd /tmp && export TMPDIR=/tmp
for r in ${ROUNDS:-1 2}; do
  for p in ${PIPES:-1 2 4}; do
    CV_BW_PIPE=$p SHAPE=c4 ITERS=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p$p.$r -o kt \
      -- python3 $R/tools/bench_fit.py > $O/p$p.$r.log 2>&1 || { echo "FAIL pipe $p"; tail -5 $O/p$p.$r.log; exit 1; }
    python3 - $O/p$p.$r $p $r <<'PY' | tee -a $O/summary.txt
import csv, glob, os, sys
rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
ends = [e for s, e, k in rows if "bw_mstep_pa" in k]
d = sorted((ends[i + 1] - ends[i]) / 1e6 for i in range(len(ends) - 1))
busy = {}
for s, e, k in rows:
    if "bw_" in k and "mstep" not in k:
        n = k.split("(")[0].replace("void cvf::", "").replace("cvf::", "")
        busy.setdefault(n, []).append((e - s) / 1e6)
print(f"pipe {sys.argv[2]} round {sys.argv[3]}: EM iteration span min {d[0]:.1f} ms (spans {' '.join(f'{x:.1f}' for x in d[:4])}); "
      + "; ".join(f"{n} x{len(v)} mean {sum(v) / len(v):.1f}" for n, v in sorted(busy.items())))
PY
    grep '"train"' $O/p$p.$r.log | cut -c1-200
  done
done
