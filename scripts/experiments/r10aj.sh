#!/bin/bash
# r10aj: MoE 128-row expert tiles of 7 waves (224 columns: 1024 live gate/up workgroups = 4 full rounds at Mixtral mb256,
# GEMM4_NW=7) vs 8 waves (896 = 3.5 rounds): MoE oracle tests with the knob, moe_bench, Mixtral engine A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
MIPIPE_GEMM4_NW=7 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_moe_gemm_gpu.py > $O/r10aj_t.log 2>&1 || { tail -30 $O/r10aj_t.log; exit 1; }
tail -1 $O/r10aj_t.log
timeout -k 10 200 python tools/moe_bench.py --M 256,512 --knob GEMM4_NW=0,7,0,7 > $O/r10aj_mb.log 2>&1 || { tail -5 $O/r10aj_mb.log; exit 1; }
grep phase $O/r10aj_mb.log
for rep in 1 2; do
  for v in 0 7; do
    MIPIPE_GEMM4_NW=$v timeout -k 10 300 python bench.py --model mixtral-8x7b --ftype Q4_K_M --steps 10 --warmup 3 --no-secondary > $O/r10aj_mx.log 2>&1 || { tail -5 $O/r10aj_mx.log; exit 1; }
    echo "rep $rep mixtral mb256 GEMM4_NW=$v $(grep -o '"value": [0-9.]*' $O/r10aj_mx.log)"
  done
done
