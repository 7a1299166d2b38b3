#!/bin/bash
# int8_gemm with split-K partial stores (deferred into the RMSNorm) vs int8 atomics: tests + A/B
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gemm_i8_gpu.py tests/test_engine_gpu.py -q -x -s -k "i8 or int8 or 70b_width" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_i8.log 2>&1; rc=$?
grep -E "int8_gemm NMSE|passed|failed" $O/t_i8.log | tail -3
[ $rc -ne 0 ] && exit $rc
for args in "" "--model llama3-8b --ftype Q4_K_M"; do
  for sk in false true false true; do
    timeout -k 10 300 python bench.py --steps 15 --warmup 3 --no-secondary $args --set int8_gemm=true --set gemm_splitk_store=$sk > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "[$args] int8 splitk_store=$sk $(grep -o '"value": [0-9.]*' $O/b.log)"
  done
done
