#!/bin/bash
# A/B over tools/bench_configs.py configs: library builds (VARIANTS="old new", tools/_ab/lib_<v>.so)
# x env settings (ENVS="CV_X=0 CV_X=1"; default none), interleaved on ONE box, ROUNDS rounds.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-abcfg}
mkdir -p $OUT
cd $R
LIB=consistent-viterbi_amd/cviterbi/libcviterbi.so
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-intree}; do
    if [ "$v" = intree ]; then unset CV_LIB_PATH; else export CV_LIB_PATH=$(pwd)/tools/_ab/lib_$v.so; fi
    for e in ${ENVS:-NONE=0}; do
      env $e REPS=${REPS:-10} timeout -k 10 ${T_CFG:-300} python tools/bench_configs.py ${CONFIGS:-c2f64 c3f64} > $OUT/$v.$e.$r.log 2>/dev/null \
        || { echo "FAIL $v $e"; exit 1; }
      python3 -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); t=d['last_call_timing']
        print(sys.argv[2], sys.argv[3], sys.argv[4], d['config'], round(d['ms_per_decode'],3), 'fwd', round(t.get('fwd_ms',0),3), 'bt', round(t.get('bt_ms',0),3))
" $OUT/$v.$e.$r.log $v $e $r | tee -a $OUT/summary.txt
    done
  done
done
