#!/bin/bash
# Round-6 GPU session driver: named steps, each under its own time limit, chained so that the
# first failure ends the call.  STEPS selects them (default: roof chain c2):
#   roof   tools/microbench/valu_roof_f64.hip: the f64 VALU roof per SIMD at 1-4 waves/SIMD
#   chain  the config-4-sized gpu-cp chain: CV_TRACE phase stamps + a kernel / copy trace
#   c2     bench_configs c2f64 (and c3f64)
#   tests  the full GPU suite;  smoke  __graft_entry__.smoke();  bench  bench.py
#   prof   rocprofv3 --kernel-trace --stats of bench.py
#   c5     bench_configs c5
# TAG names the output directory under gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r06_s1}
mkdir -p $O
cd $R
export TMPDIR=/tmp
step() {
  local name=$1 t=$2
  shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  tail -4 $O/$name.log | cut -c1-300
  echo "== $name rc=$rc"
  return $rc
}
run() {
  case $1 in
    roof)
      hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_roof_f64 tools/microbench/valu_roof_f64.hip > $O/roof_build.log 2>&1 &&
        step roof 180 /tmp/valu_roof_f64 ;;
    chain)
      CV_TRACE=1 step chain_phases 240 python3 -u tools/bench_chain.py 65536 256 &&
        (cd /tmp && SERIAL=0 step chain_trace 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
          -d $O/kt -o kt -- python3 $R/tools/bench_chain_large_n.py 256 256 65536) &&
        python3 tools/trace_timeline.py $O/kt trellis_fwd_f64 > $O/chain_timeline.txt ;;
    c2) REPS=20 step c2 200 python3 -u tools/bench_configs.py c2f64 c3f64 ;;
    c2ab) REPS=50 step c2ab_on 200 python3 -u tools/bench_configs.py c2f64 &&
      REPS=50 CV_T64_BAL=0 step c2ab_off 200 python3 -u tools/bench_configs.py c2f64 &&
      REPS=50 CV_T64_WAVE=2 step c2ab_w64 200 python3 -u tools/bench_configs.py c2f64 ;;
    c5) step c5 300 python3 -u tools/bench_configs.py c5 ;;
    tests) step tests 900 python3 -u -m pytest -q --maxfail=25 --timeout 200 --timeout-method thread -m gpu tests ;;
    chainq) step chainq 240 python3 -u tools/bench_chain.py 65536 256 ;;
    chainab)  # the speculative batch's kernel: generic / trellis_cp_f64 split columns (S, rows in flight)
      step chainab_gen 240 python3 -u tools/bench_chain.py 65536 256 &&
        CV_CHAIN_SPEC_KERNEL=1 step chainab_cp4 240 python3 -u tools/bench_chain.py 65536 256 &&
        CV_CHAIN_SPEC_KERNEL=1 CV_T64_CP_PF=16 step chainab_cp4pf16 240 python3 -u tools/bench_chain.py 65536 256 &&
        CV_CHAIN_SPEC_KERNEL=1 CV_T64_CP_S=2 step chainab_cp2 240 python3 -u tools/bench_chain.py 65536 256 &&
        (cd /tmp && CV_CHAIN_SPEC_KERNEL=1 SERIAL=0 step chainab_trace 300 rocprofv3 --kernel-trace --memory-copy-trace \
          --output-format csv -d $O/kt -o kt -- python3 $R/tools/bench_chain_large_n.py 256 256 65536) &&
        python3 tools/trace_timeline.py $O/kt trellis_fwd_f64 > $O/chain_timeline.txt ;;
    chaintests) step chaintests 600 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread -m gpu \
      tests/test_gpu_chain_par.py tests/test_gpu_f64.py -k "chain or cp_seqs or wave48" ;;
    w48t) step w48t 400 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread -m gpu \
      tests/test_gpu_f64.py tests/test_gpu_configs_oracle.py -k "wave48 or c2 or golden or wave" ;;
    c2pmc)  # where trellis_wave48_f64's waves spend their cycles
      (cd /tmp && REPS=3 step c2pmc1 120 rocprofv3 --kernel-include-regex wave48 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -d $O/pmc1 -o pmc1 --output-format csv \
        -- python3 $R/tools/bench_configs.py c2f64) &&
      (cd /tmp && REPS=3 step c2pmc2 120 rocprofv3 --kernel-include-regex wave48 --pmc SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY \
        SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $O/pmc2 -o pmc2 --output-format csv \
        -- python3 $R/tools/bench_configs.py c2f64) ;;
    spec) step spec 300 python3 -u tools/bench_spec.py 573 143 64 ;;
    specu16) CV_LIB_PATH=$R/tools/_ab/libcv_u16.so step specu16 300 python3 -u tools/bench_spec.py 573 143 ;;
    btpf)  # the backtrack's rows in flight (tuning key t64_bt_pf): config 4 and the chain
      for pf in 2 4 8; do
        REPS=3 CV_T64_BT_PF=$pf step btpf_c4_$pf 200 python3 -u tools/bench_configs.py c4f64 &&
          CV_T64_BT_PF=$pf step btpf_chain_$pf 240 python3 -u tools/bench_chain.py 65536 256 || return $?
      done ;;
    btab)  # block-refilled vs rolling backtrack row ring, rows in flight 2 / 4 / 8 (config 4)
      for pf in 2 4 8; do
        REPS=3 CV_T64_BT_PF=$pf step btab_main_$pf 200 python3 -u tools/bench_configs.py c4f64 &&
          REPS=3 CV_T64_BT_PF=$pf CV_LIB_PATH=$R/tools/_ab/libcv_roll.so step btab_roll_$pf 200 \
            python3 -u tools/bench_configs.py c4f64 || return $?
      done ;;
    smoke) step smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    bench) step bench 400 python3 -u bench.py ;;
    prof)
      (cd /tmp && step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- python3 $R/bench.py --no-f32-extra) ;;
    *) echo "unknown step $1"; return 2 ;;
  esac
}
for s in ${STEPS:-roof chain c2}; do
  run $s || exit $?
done
