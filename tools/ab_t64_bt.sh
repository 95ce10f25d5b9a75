set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "f64 or t64" --timeout 120 --timeout-method thread > gpurun_out/ab/pytest_f64.log 2>&1 || { tail -20 gpurun_out/ab/pytest_f64.log; exit 1; }
tail -2 gpurun_out/ab/pytest_f64.log
for pf in ${PFS:-4 8 16}; do
  CV_T64_BT_PF=$pf timeout -k 10 300 python bench.py --dtype f64 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/ab/bench_pf$pf.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab/bench_pf$pf.log').read().strip().splitlines()[-1]); print($pf, d['ms_per_step'], d['kernel_ms_per_step'])"
done
