#!/bin/bash
# A/B: generic_fwd_ms<4>'s psi walk rolled (base) vs unrolled (u4, -DCVK_GEN_UNROLL_S=4), on the
# config-4-sized chain's speculative batch (CV_GENERIC_S=4 vs the default S = 2) and on a large
# psi-mode batch (CP, N = 300, 8,192 x 128, S = 4 by default); interleaved on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_unroll_s4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for r in 1 2; do
  for v in base u4; do
    export CV_LIB_PATH=$R/tools/_ab/lib_$v.so
    for s in 4 2; do
      CV_GENERIC_S=$s SERIAL=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$v$s.$r -o kt -- python3 $R/tools/bench_chain_large_n.py 256 256 65536 > $OUT/chain$v$s.$r.log 2>&1 || { tail -5 $OUT/chain$v$s.$r.log; exit 1; }
      python3 - $OUT/kt$v$s.$r/kt_kernel_stats.csv "$v S=$s round $r" <<'PY' | tee -a $OUT/summary.txt
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    if "generic_fwd" in row["Name"]:
        print(f"chain spec {sys.argv[2]}: {row['Name'].split('(')[0][-40:]} {float(row['AverageNs']) / 1e6:.2f} ms x{row['Calls']}")
PY
    done
    timeout -k 10 300 python3 - $R "$v round $r" <<'PY' | tee -a $OUT/summary.txt
import sys, time
sys.path.insert(0, sys.argv[1] + "/consistent-viterbi_amd")
import numpy as np
import cviterbi as cv
from cviterbi import synth
n, nseq, T = 300, 8192, 128
pi, a, b = synth.random_hmm(n, 64, seed=n)
off = synth.offsets_from_lengths(np.full(nseq, T))
obs = synth.iid_obs(64, nseq * T, n)
h = cv.HMM(pi, a, b)
ref = cv.decode_batch(h, off, obs, dtype="f64", assoc="cp", kernel="generic", rescore_f64=False)
t0 = time.perf_counter()
for _ in range(3):
    got = cv.decode_batch(h, off, obs, dtype="f64", assoc="cp", kernel="generic", rescore_f64=False)
dt = (time.perf_counter() - t0) / 3
print(f"psi CP N=300 8192x128 {sys.argv[2]}: {dt * 1e3:.1f} ms, fwd {cv.last_timing(h)['fwd_ms']:.1f} ms, same={all(np.array_equal(x, y) for x, y in zip(ref, got))}")
PY
  done
done
