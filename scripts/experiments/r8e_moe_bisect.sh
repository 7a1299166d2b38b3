#!/bin/bash
# r8e: bisect the grouped-MoE down-projection mismatch (Mixtral widths): row tile x split-K x weight type
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 300 python -u -m pytest -q --timeout 250 --timeout-method thread -m gpu -p no:cacheprovider tests/test_moe_gemm_gpu.py -k mixtral"
for cfg in "" "" "MIPIPE_GEMM3_SPLIT=2" "MIPIPE_GEMM3_SPLIT=4" "MOE_TEST_DOWN_QT=12" "MOE_TEST_DOWN_QT=12 MIPIPE_GEMM3_SPLIT=1" "MIPIPE_GEMM3_BM=128 MIPIPE_GEMM3_SPLIT=4"; do
  env $cfg $T > $O/r8e.log 2>&1; rc=$?
  echo "[$cfg] rc=$rc $(grep -E 'passed|failed' $O/r8e.log | tail -1) $(grep -E '^FAILED' $O/r8e.log | sed 's/.*\[//' | tr '\n' ' ') $(grep -o 'assert [0-9.e-]* < 1e-0[45]' $O/r8e.log | tr '\n' ' ')"
  [ $rc -gt 1 ] && exit $rc
done
exit 0
