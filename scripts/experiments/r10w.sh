#!/bin/bash
# r10w: MoE down K splits (GEMM3_SPLIT forces the split count of the MoE down: 0 = auto = unsplit at 128-row tiles):
# moe_bench at M = 256 / 512, then the engine at Mixtral mb256 with the best candidates
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
timeout -k 10 300 python tools/moe_bench.py --M 256,512 --phases down --knob GEMM3_SPLIT=0,2,3,4,5,6,7,8 > $O/r10w_mb.log 2>&1 || { tail -5 $O/r10w_mb.log; exit 1; }
grep phase $O/r10w_mb.log
