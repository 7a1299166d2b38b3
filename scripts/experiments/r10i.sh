#!/bin/bash
# r10i: 64-row micro-batches on gemm4 (knob GEMM4_M64) -- oracle tests, engine test, 70B / 8B mb64 A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemm4_gpu.py -k "64_row" > $O/r10i_t.log 2>&1 || { tail -30 $O/r10i_t.log; exit 1; }
tail -1 $O/r10i_t.log
MIPIPE_GEMM4_M64=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_engine_gpu.py -k "wide_microbatch" > $O/r10i_t2.log 2>&1 || { tail -30 $O/r10i_t2.log; exit 1; }
tail -1 $O/r10i_t2.log
for rep in 1 2; do
  for v in 0 1; do
    MIPIPE_GEMM4_M64=$v timeout -k 10 300 python bench.py --mb-size 64 --steps 10 --warmup 3 --no-secondary > $O/r10i_70b_$v.log 2>&1 || { tail -5 $O/r10i_70b_$v.log; exit 1; }
    echo "rep $rep 70b mb64 GEMM4_M64=$v $(grep -o '"value": [0-9.]*' $O/r10i_70b_$v.log)"
  done
done
for v in 0 1; do
  MIPIPE_GEMM4_M64=$v timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 64 --steps 10 --warmup 3 --no-secondary > $O/r10i_8b_$v.log 2>&1 || exit 1
  echo "8b mb64 GEMM4_M64=$v $(grep -o '"value": [0-9.]*' $O/r10i_8b_$v.log)"
  MIPIPE_GEMM4_M64=$v timeout -k 10 300 python bench.py --model mixtral-8x7b --ftype Q4_K_M --mb-size 64 --steps 10 --warmup 3 --no-secondary > $O/r10i_mx_$v.log 2>&1 || exit 1
  echo "mixtral mb64 GEMM4_M64=$v $(grep -o '"value": [0-9.]*' $O/r10i_mx_$v.log)"
done
