#!/bin/bash
# Forward/backtrack times of library variants (tools/_ab/lib_<v>.so, tools/build_variant.sh) at
# several batch sizes, interleaved on ONE box, via tools/bench_assoc.py (timing only: ablation
# variants decode wrong results).  VARIANTS="base x" NSEQS="8192 65536" ROUNDS=2 tools/ab_lib_fwd.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-abfwd}
mkdir -p $OUT
cd $R
LIB=consistent-viterbi_amd/cviterbi/libcviterbi.so
for r in $(seq 1 ${ROUNDS:-2}); do
  for n in ${NSEQS:-8192 65536}; do
    for v in ${VARIANTS:-base}; do
      export CV_LIB_PATH=$(pwd)/tools/_ab/lib_$v.so
      NSEQ=$n timeout -k 10 ${T_BENCH:-120} python tools/bench_assoc.py ${ASSOC:-viterbi} > $OUT/$v.$n.$r.log 2>&1 || { echo "FAIL $v $n"; tail -5 $OUT/$v.$n.$r.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], sys.argv[4], 'ms', round(d['ms'],3), 'fwd', round(d['fwd_ms'],3), 'bt', round(d['bt_ms'],3))" $OUT/$v.$n.$r.log $v $n $r | tee -a $OUT/summary.txt
    done
  done
done
