#!/bin/bash
# r10v: MoE grouped GEMM with 4 waves x 64 columns at 128-row expert tiles (GEMM4_TW4=3) vs the 8-wave form (1):
# MoE oracle tests with the knob, moe_bench, Mixtral mb256 / mb64 engine A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
MIPIPE_GEMM4_TW4=3 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_moe_gemm_gpu.py > $O/r10v_t.log 2>&1 || { tail -30 $O/r10v_t.log; exit 1; }
tail -1 $O/r10v_t.log
timeout -k 10 200 python tools/moe_bench.py --M 256,64 --knob GEMM4_TW4=1,3 > $O/r10v_mb.log 2>&1 || { tail -5 $O/r10v_mb.log; exit 1; }
cat $O/r10v_mb.log
for rep in 1 2; do
  for v in 1 3; do
    MIPIPE_GEMM4_TW4=$v timeout -k 10 300 python bench.py --model mixtral-8x7b --ftype Q4_K_M --steps 10 --warmup 3 --no-secondary > $O/r10v_mx_$v.log 2>&1 || { tail -5 $O/r10v_mx_$v.log; exit 1; }
    echo "rep $rep mixtral mb256 GEMM4_TW4=$v $(grep -o '"value": [0-9.]*' $O/r10v_mx_$v.log)"
  done
done
