#!/bin/bash
# r10ag: the LM head (Q6_K, 128256 x 8192, M = 256, 256-row tiles) with the 4-wave form (GEMM4_TW4=1) vs 8 waves (0)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
timeout -k 10 300 python tools/gemv_bench.py --M 256 --iters 12 --gemm 4 --shapes 70b.head --knob GEMM4_TW4=0,1,0,1,0,1 > $O/r10ag.log 2>&1 || { tail -5 $O/r10ag.log; exit 1; }
grep -o '"shape": "[^"]*".*"us": [0-9.]*.*"knobs": {[^}]*}' $O/r10ag.log | sed 's/"type.*"us"/ us/; s/"GBps.*"knobs"/ knobs/'
b8() { timeout -k 10 200 env "$@" python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 32 --warmup 4 --no-secondary > $O/r10ag_8b.log 2>&1 || { tail -3 $O/r10ag_8b.log; exit 1; }; echo "8b mb1 $* $(grep -o '"value": [0-9.]*' $O/r10ag_8b.log)"; }
b8 X=0
for v in 1 2 4 8; do b8 MIPIPE_GEMVS_G=$v; done
for v in 2 4; do b8 MIPIPE_GEMVS_SPLIT=$v; done
b8 X=0
