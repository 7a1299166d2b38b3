#!/bin/bash
# r10n: gemm4 128-row tiles with a 4-stage LDS ring (lib_b) against the 3-stage default, same box
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
MIPIPE_LIB=../lib_b/libmipipe.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gemm4_gpu.py > $O/r10n_t.log 2>&1 || { tail -30 $O/r10n_t.log; exit 1; }
tail -1 $O/r10n_t.log
for lib in libmipipe.so ../lib_b/libmipipe.so; do
  MIPIPE_LIB=$lib timeout -k 10 200 python tools/gemv_bench.py --M 256 --iters 24 --gemm 4 --sk --shapes 70b.qkv,70b.o,70b.down,8b.qkv,8b.down > $O/r10n_gb.log 2>&1 || { tail -5 $O/r10n_gb.log; exit 1; }
  echo "$lib"; grep -o '"shape": "[^"]*".*"us": [0-9.]*' $O/r10n_gb.log | sed 's/"type.*"us"/ us/'
done
for rep in 1 2; do
  for lib in libmipipe.so ../lib_b/libmipipe.so; do
    MIPIPE_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-secondary > $O/r10n_70b.log 2>&1 || { tail -5 $O/r10n_70b.log; exit 1; }
    echo "rep $rep 70b mb256 $lib $(grep -o '"value": [0-9.]*' $O/r10n_70b.log)"
  done
done
