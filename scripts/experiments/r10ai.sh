#!/bin/bash
# r10ai: gemm4 timing probes on the MoE gate/up (probe library): Mixtral widths, M = 256 tokens (top-2 of 8), 128-row
# expert tiles, with the dequant / MFMA / LDS-DMA parts skipped in every combination
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
export MIPIPE_LIB=../lib_probe/libmipipe.so
for rep in 1 2; do
  timeout -k 10 200 python tools/moe_bench.py --M 256 --phases gateup --knob GEMM4_PROBE=0,1,2,3,4,5,6,7 > $O/r10ai_$rep.log 2>&1 || { tail -5 $O/r10ai_$rep.log; exit 1; }
  echo "pass $rep"; grep phase $O/r10ai_$rep.log
done
