#!/bin/bash
# Round 5 session 7: where the f32 pair trellis's time goes -- timing-only ablation builds
# (tools/build_variant_f32.sh: CVK_F32_ABL_OBS / NOE / NOSTORE) interleaved on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ABTAG:-r05_s7}
mkdir -p $O
cd $R
for r in 1 2; do
  for v in ${VARIANTS:-new aobs anoe anost aall}; do
    CV_LIB_PATH=$R/tools/_ab/lib_$v.so timeout -k 10 240 python bench.py --dtype f32 --steps 8 --warmup 2 --no-cpu-baseline \
      --no-f32-extra --no-configs > $O/$v.$r.log 2>&1 || { echo "FAIL $v"; tail -5 $O/$v.$r.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],2), 'fwd', round(d['kernel_ms_per_step']['forward'],2))" $O/$v.$r.log $v $r | tee -a $O/summary.txt
  done
done
