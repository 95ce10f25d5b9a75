#!/bin/bash
# The parallel chain's GPU tests, then interleaved A/B of the config-4-sized solve over tuning
# keys (VARIANTS: space-free env assignments joined by commas, ";"-separated).  Output under
# gpurun_out/${TAG:-ab_chain}.
O=gpurun_out/${TAG:-ab_chain}
mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_chain_par.py \
    > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || exit $rc
fi
IFS=';' read -ra VS <<< "${VARIANTS:-;CV_CHAIN_PIN_OBS=0,CV_CHAIN_PIN_PATH=0;CV_CHAIN_PIN_PATH=0}"
for rep in 1 2; do
  for v in "${VS[@]}"; do
    echo "== ${v:-default}"
    env ${v//,/ } timeout -k 10 200 python3 -u tools/chain_reps.py 2>&1 | grep "chain ms" || exit 1
  done
done
