#!/bin/bash
# r10k: gemm4 fragment schedule A/B (lib_b: B fragment t+1 right behind fragment t's first MFMA,
# next-stage prep three steps after its raw reads) against the default library, same box
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
export MIPIPE_LIB_B=../lib_b/libmipipe.so
MIPIPE_LIB=$MIPIPE_LIB_B timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gemm4_gpu.py tests/test_moe_gemm_gpu.py > $O/r10k_t.log 2>&1 || { tail -30 $O/r10k_t.log; exit 1; }
tail -1 $O/r10k_t.log
for lib in libmipipe.so ../lib_b/libmipipe.so; do
  MIPIPE_LIB=$lib timeout -k 10 200 python tools/gemv_bench.py --M 256 --iters 24 --gemm 4 --sk --shapes 70b.gateup,70b.qkv,70b.down > $O/r10k_gb.log 2>&1 || { tail -5 $O/r10k_gb.log; exit 1; }
  echo "$lib"; grep -o '"shape": "[^"]*".*"us": [0-9.]*' $O/r10k_gb.log | sed 's/"type.*"us"/ us/'
done
for rep in 1 2; do
  for lib in libmipipe.so ../lib_b/libmipipe.so; do
    MIPIPE_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-secondary > $O/r10k_70b.log 2>&1 || { tail -5 $O/r10k_70b.log; exit 1; }
    echo "rep $rep 70b mb256 $lib $(grep -o '"value": [0-9.]*' $O/r10k_70b.log)"
    MIPIPE_LIB=$lib timeout -k 10 300 python bench.py --model mixtral-8x7b --ftype Q4_K_M --steps 10 --warmup 3 --no-secondary > $O/r10k_mx.log 2>&1 || { tail -5 $O/r10k_mx.log; exit 1; }
    echo "rep $rep mixtral mb256 $lib $(grep -o '"value": [0-9.]*' $O/r10k_mx.log)"
  done
done
