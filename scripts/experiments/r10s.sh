#!/bin/bash
# r10s: gemm4 timing probes (probe library): 70B gate/up at M = 256 (SwiGLU, 256-row tiles) and the 70B down split-K
# store (128-row tiles) with the dequant / MFMA / LDS-DMA parts skipped in every combination (GEMM4_PROBE bits 0-2)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
export MIPIPE_LIB=../lib_probe/libmipipe.so
for rep in 1 2; do
  timeout -k 10 200 python tools/gemv_bench.py --M 256 --iters 24 --gemm 4 --shapes 70b.gateup --knob GEMM4_PROBE=0,1,2,3,4,5,6,7 > $O/r10s_gu_$rep.log 2>&1 || { tail -5 $O/r10s_gu_$rep.log; exit 1; }
  echo "gateup pass $rep"; grep -o '"us": [0-9.]*.*"knobs": {[^}]*}' $O/r10s_gu_$rep.log | sed 's/"GBps.*"knobs"/ knobs/'
  timeout -k 10 200 python tools/gemv_bench.py --M 256 --iters 24 --gemm 4 --sk --shapes 70b.down,70b.qkv --knob GEMM4_PROBE=0,1,2,3,4,5,6,7 > $O/r10s_dn_$rep.log 2>&1 || { tail -5 $O/r10s_dn_$rep.log; exit 1; }
  echo "down/qkv pass $rep"; grep -o '"shape": "[^"]*".*"us": [0-9.]*.*"knobs": {[^}]*}' $O/r10s_dn_$rep.log | sed 's/"type.*"us"/ us/; s/"GBps.*"knobs"/ knobs/'
done
