#!/bin/bash
# Round 5 session 2: the full GPU suite at HEAD, the parallel chain at N = 1,024 (4,096 x 512 vs
# the serial chain) and at config-4 size (N = 512, 65,536 x 512), the MFMA microbench rerun,
# and the 8-rank gloo rehearsal of the driver's SCALE command (collective pre-flight).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_s2
mkdir -p $O
cd $R
step() {  # name, timeout, command...: output straight into a file under gpurun_out (no pipe)
  local name=$1 t=$2
  shift 2
  echo "== $name" ; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  tail -4 $O/$name.log; echo "== $name rc=$rc"; return $rc
}
step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread &&
step chain_1024 600 python -u tools/bench_chain_large_n.py 1024 4096 &&
step chain_512_c4 300 python -u tools/bench_chain_large_n.py 512 2048 65536 &&
step mfma 120 tools/microbench/mfma_f64_coissue &&
step rehearsal_8rank 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 8 --backend gloo --steps 2 --warmup 1 --no-cpu-baseline --no-f32-extra --no-configs
