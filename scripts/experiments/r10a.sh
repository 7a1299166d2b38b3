#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm4_gpu.py tests/test_moe_gemm_gpu.py tests/test_gemm3_gpu.py > $O/r10a_t.log 2>&1; rc=$?
tail -5 $O/r10a_t.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-secondary > $O/r10a_b1.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' $O/r10a_b1.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-secondary --set prefill_gemm_v=4 > $O/r10a_b2.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' $O/r10a_b2.log
