# f64 backtrack rows in flight (CV_T64_BT_PF) at NP = 64 (configs 2 and 3); bit-identical knob
set -o pipefail
mkdir -p gpurun_out/ab
for pf in 2 4 8 2 8; do
  CV_T64_BT_PF=$pf timeout -k 10 300 python tools/bench_configs.py c2f64 c3f64 > gpurun_out/ab/small_pf$pf.log 2>&1 || exit 1
  python -c "
import json
for l in open('gpurun_out/ab/small_pf$pf.log'):
    if l.startswith('{'):
        d = json.loads(l); print($pf, d['config'], round(d['ms_per_decode'], 4), round(d['last_call_timing']['bt_ms'], 4))"
done
