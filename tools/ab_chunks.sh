# f32 config-4 pipeline depth (CV_MAX_CHUNKS, bit-identical knob): ms/step and kernel ms/step
set -o pipefail
mkdir -p gpurun_out/ab
for c in ${CHUNKS:-8 12 16 8 16}; do
  CV_MAX_CHUNKS=$c timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/ab/chunks_$c.log 2>&1 || exit 1
  python -c "import json; d=json.loads([l for l in open('gpurun_out/ab/chunks_$c.log') if l.startswith('{')][-1]); print($c, d['ms_per_step'], d['kernel_ms_per_step'])"
done
