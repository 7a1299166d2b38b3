#!/bin/bash
# r10x: 128-row gemm4 tiles of 4 waves, two workgroups per CU (GEMM4_NW=4) -- oracle tests with the knob, split-K
# shapes micro-bench, engine A/B at 70B / 8B mb256 and Mixtral (its qkv / o)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
MIPIPE_GEMM4_NW=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gemm4_gpu.py > $O/r10x_t.log 2>&1 || { tail -30 $O/r10x_t.log; exit 1; }
tail -1 $O/r10x_t.log
timeout -k 10 300 python tools/gemv_bench.py --M 256 --iters 24 --gemm 4 --sk --shapes 70b.qkv,70b.o,70b.down,8b.qkv,8b.down --knob GEMM4_NW=0,4,0,4 > $O/r10x_sk.log 2>&1 || { tail -5 $O/r10x_sk.log; exit 1; }
grep -o '"shape": "[^"]*".*"us": [0-9.]*.*"knobs": {[^}]*}' $O/r10x_sk.log | sed 's/"type.*"us"/ us/; s/"GBps.*"knobs"/ knobs/'
for rep in 1 2; do
  for v in 0 4; do
    MIPIPE_GEMM4_NW=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-secondary > $O/r10x_70b_$v.log 2>&1 || { tail -5 $O/r10x_70b_$v.log; exit 1; }
    echo "rep $rep 70b mb256 GEMM4_NW=$v $(grep -o '"value": [0-9.]*' $O/r10x_70b_$v.log)"
  done
done
for v in 0 4; do
  MIPIPE_GEMM4_NW=$v timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --steps 10 --warmup 3 --no-secondary > $O/r10x_8b_$v.log 2>&1 || { tail -5 $O/r10x_8b_$v.log; exit 1; }
  echo "8b mb256 GEMM4_NW=$v $(grep -o '"value": [0-9.]*' $O/r10x_8b_$v.log)"
done
