#!/bin/bash
# r10q: split-K decode projections at M = 256 per shape: gemm2 (gemv2 128x256 tiles) vs gemm4 (32x32x16 MFMA), cold weights
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
for g in 2 4; do
  timeout -k 10 200 python tools/gemv_bench.py --M 256,128 --iters 24 --gemm $g --sk --shapes 70b.qkv,70b.o,70b.down,8b.qkv,8b.o,8b.down > $O/r10q_g$g.log 2>&1 || { tail -5 $O/r10q_g$g.log; exit 1; }
  echo "gemm $g"; grep -o '"shape": "[^"]*".*"M": [0-9]*.*"us": [0-9.]*' $O/r10q_g$g.log | sed 's/"type.*"M"/ M/; s/"tpw.*"us"/ us/'
done
