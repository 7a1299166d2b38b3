#!/bin/bash
# r8z: gemm4 MoE mode skips the MFMAs of 32-row fragments past an expert's routed rows (Mixtral at
# 256 tokens: ~64 rows per expert in 128-row tiles): tests, then Mixtral A/B against the r8y build
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 600 python -u -m pytest -q --timeout 250 --timeout-method thread -m gpu -p no:cacheprovider"
$T tests/test_moe_gemm_gpu.py tests/test_gemm4_gpu.py > $O/r8z_t.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" $O/r8z_t.log | tail -4; [ $rc -ne 0 ] && exit $rc
$T tests/test_engine_gpu.py -k "moe or mixtral" > $O/r8z_t2.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" $O/r8z_t2.log | tail -4; [ $rc -ne 0 ] && exit $rc
BB="timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-secondary --model mixtral-8x7b --ftype Q4_K_M"
for rep in 1 2; do for lib in new old; do
  if [ $lib = old ]; then export MIPIPE_LIB=libmipipe_old.so; else unset MIPIPE_LIB; fi
  $BB > $O/r8z_mx_$lib.log 2>&1 || { tail -3 $O/r8z_mx_$lib.log; exit 1; }
  echo "rep $rep $lib: mixtral mb256 $(grep -o '"value": [0-9.]*' $O/r8z_mx_$lib.log)"
done; done
unset MIPIPE_LIB
$BB --mb-size 64 > $O/r8z_mx64.log 2>&1 || exit 1; echo "mixtral mb64 new $(grep -o '"value": [0-9.]*' $O/r8z_mx64.log)"
