cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r06_bwab
for v in base nobnum norows noalpha; do
  if [ $v = base ]; then unset CV_LIB_PATH; else export CV_LIB_PATH=$R/tools/_ab/lib_$v.so; fi
  SHAPE=c4 BATCH=16384 ITERS=2 MODES=train timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r06_bwab/$v -o s -- python3 $R/tools/bench_fit.py train > $R/gpurun_out/r06_bwab/$v.log 2>&1 || exit 1
  echo "== $v"; grep -h "bw_fwd_mm\|bw_bwd_mm\|bw_xi_gemm" $R/gpurun_out/r06_bwab/$v/s_kernel_stats.csv | cut -d, -f1-5 | sed 's/(cvk::BwArgs[^"]*//' | cut -c1-120
done
