#!/bin/bash
# r10r: gemm4 split-K decode projections at M = 256: rows per workgroup (GEMM3_BM 0 = auto, 128, 256) x splits
# (GEMM3_SPLIT 0 = auto), two passes (the box drifts a few % over a minute)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
for rep in 1 2; do
  timeout -k 10 300 python tools/gemv_bench.py --M 256 --iters 24 --gemm 4 --sk --shapes 70b.qkv,70b.o,70b.down,8b.down --knob GEMM3_BM=0,128,256 --knob GEMM3_SPLIT=0,2,4,8 > $O/r10r_$rep.log 2>&1 || { tail -5 $O/r10r_$rep.log; exit 1; }
  echo "pass $rep"; grep -o '"shape": "[^"]*".*"us": [0-9.]*.*"knobs": {[^}]*}' $O/r10r_$rep.log | sed 's/"type.*"us"/ us/; s/"GBps.*"knobs"/ knobs/'
done
