#!/bin/bash
# r10t: gemm4 dense with 4 waves x 64 columns (knob GEMM4_TW4: two MFMAs per LDS A fragment, one wave per SIMD, 512
# registers) -- oracle tests with the knob on, micro-bench of the 70B shapes, engine A/B at 70B / 8B mb256
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
MIPIPE_GEMM4_TW4=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gemm4_gpu.py > $O/r10t_t.log 2>&1 || { tail -30 $O/r10t_t.log; exit 1; }
tail -1 $O/r10t_t.log
timeout -k 10 200 python tools/gemv_bench.py --M 256 --iters 24 --gemm 4 --shapes 70b.gateup --knob GEMM4_TW4=0,1,0,1 > $O/r10t_gu.log 2>&1 || { tail -5 $O/r10t_gu.log; exit 1; }
grep -o '"shape": "[^"]*".*"us": [0-9.]*.*"knobs": {[^}]*}' $O/r10t_gu.log | sed 's/"type.*"us"/ us/; s/"GBps.*"knobs"/ knobs/'
timeout -k 10 200 python tools/gemv_bench.py --M 256 --iters 24 --gemm 4 --sk --shapes 70b.qkv,70b.o,70b.down --knob GEMM4_TW4=0,1,0,1 > $O/r10t_sk.log 2>&1 || { tail -5 $O/r10t_sk.log; exit 1; }
grep -o '"shape": "[^"]*".*"us": [0-9.]*.*"knobs": {[^}]*}' $O/r10t_sk.log | sed 's/"type.*"us"/ us/; s/"GBps.*"knobs"/ knobs/'
for rep in 1 2; do
  for v in 0 1; do
    MIPIPE_GEMM4_TW4=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-secondary > $O/r10t_70b_$v.log 2>&1 || { tail -5 $O/r10t_70b_$v.log; exit 1; }
    echo "rep $rep 70b mb256 GEMM4_TW4=$v $(grep -o '"value": [0-9.]*' $O/r10t_70b_$v.log)"
  done
done
