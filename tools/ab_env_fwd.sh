#!/bin/bash
# Env-knob A/B of the decode at several batch sizes via tools/bench_assoc.py (forward /
# backtrack times + a digest of the results), interleaved on ONE box:
#   AB="CV_X=0 CV_X=1" NSEQS="65536 8192" ROUNDS=2 tools/ab_env_fwd.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-abenvfwd}
mkdir -p $OUT
cd $R
for r in $(seq 1 ${ROUNDS:-2}); do
  for n in ${NSEQS:-65536}; do
    for v in $AB; do
      env $v NSEQ=$n timeout -k 10 ${T_BENCH:-120} python tools/bench_assoc.py ${ASSOC:-viterbi} > $OUT/$v.$n.$r.log 2>&1 || { echo "FAIL $v $n"; tail -5 $OUT/$v.$n.$r.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], sys.argv[4], 'ms', round(d['ms'],3), 'fwd', round(d['fwd_ms'],3), 'bt', round(d['bt_ms'],3), d['sha16'])" $OUT/$v.$n.$r.log $v $n $r | tee -a $OUT/summary.txt
    done
  done
done
