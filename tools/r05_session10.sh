#!/bin/bash
# Round 5 session 10: the parallel chain beyond N = 1,024; the driver's SCALE command rehearsed
# with 8 gloo ranks on this one GPU (collective pre-flight); the strong-scaling shard's step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_s10
mkdir -p $O
cd $R
step() {
  local name=$1 t=$2
  shift 2
  echo "== $name" ; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  tail -3 $O/$name.log | cut -c1-400; echo "== $name rc=$rc"; return $rc
}
step tests 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_chain_par.py -k beyond_1024 &&
step shard8192 240 python -u bench.py --batch 8192 --steps 20 --warmup 3 --no-cpu-baseline --no-f32-extra --no-configs &&
step shard16384 240 python -u bench.py --batch 16384 --steps 10 --warmup 2 --no-cpu-baseline --no-f32-extra --no-configs &&
step rehearsal_8rank 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 8 --backend gloo --steps 2 --warmup 1 --no-cpu-baseline --no-f32-extra --no-configs
