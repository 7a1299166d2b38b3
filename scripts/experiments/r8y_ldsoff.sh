#!/bin/bash
# r8y: LDS addresses of the DMA / LDS reads as the low half of the generic pointer (no null-checked address-space cast): tests, then engine A/B against the r8w build (lib/libmipipe_old.so)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 600 python -u -m pytest -q --timeout 250 --timeout-method thread -m gpu -p no:cacheprovider"
$T tests/test_gemm4_gpu.py tests/test_gemm3_gpu.py tests/test_moe_gemm_gpu.py > $O/r8y_t.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" $O/r8y_t.log | tail -4; [ $rc -ne 0 ] && exit $rc
$T tests/test_engine_gpu.py -k "70b or moe or mixtral or wide" > $O/r8y_t2.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" $O/r8y_t2.log | tail -4; [ $rc -ne 0 ] && exit $rc
BB="timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-secondary"
for rep in 1 2; do
for lib in new old; do
  if [ $lib = old ]; then export MIPIPE_LIB=libmipipe_old.so; else unset MIPIPE_LIB; fi
  $BB > $O/r8y_70_$lib.log 2>&1 || { tail -3 $O/r8y_70_$lib.log; exit 1; }
  $BB --model mixtral-8x7b --ftype Q4_K_M > $O/r8y_mx_$lib.log 2>&1 || { tail -3 $O/r8y_mx_$lib.log; exit 1; }
  echo "rep $rep $lib: 70b mb256 $(grep -o '"value": [0-9.]*' $O/r8y_70_$lib.log) | mixtral mb256 $(grep -o '"value": [0-9.]*' $O/r8y_mx_$lib.log)"
done; done
unset MIPIPE_LIB
$BB --model llama3-8b --ftype Q4_K_M > $O/r8y_8.log 2>&1 || exit 1; echo "8b mb256 new $(grep -o '"value": [0-9.]*' $O/r8y_8.log)"
MIPIPE_LIB=libmipipe_old.so $BB --model llama3-8b --ftype Q4_K_M > $O/r8y_8o.log 2>&1 || exit 1; echo "8b mb256 old $(grep -o '"value": [0-9.]*' $O/r8y_8o.log)"
