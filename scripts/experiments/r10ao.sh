#!/bin/bash
# r10ao: split-K decode projections at M = 256 on 256-row tiles with the 4-wave form (GEMM3_BM=256, GEMM4_TW4=1) vs the
# default 128-row 8-wave tiles, alternated twice
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
timeout -k 10 300 python tools/gemv_bench.py --M 256 --iters 24 --gemm 4 --sk --shapes 70b.qkv,70b.o,70b.down --knob GEMM3_BM=0,256,0,256 > $O/r10ao.log 2>&1 || { tail -5 $O/r10ao.log; exit 1; }
grep -o '"shape": "[^"]*".*"us": [0-9.]*.*"knobs": {[^}]*}' $O/r10ao.log | sed 's/"type.*"us"/ us/; s/"GBps.*"knobs"/ knobs/'
