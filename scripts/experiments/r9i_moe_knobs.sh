#!/bin/bash
# r9i: Mixtral mb256 vs the MoE down projection's K splits (GEMM3_SPLIT: 0 = auto (2 at 256 tokens),
# 1, 4) and non-temporal expert weights off (GEMM4_WNT=2), two interleaved reps
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
BB="timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-secondary --model mixtral-8x7b --ftype Q4_K_M"
for rep in 1 2; do
  for v in "GEMM3_SPLIT=0" "GEMM3_SPLIT=1" "GEMM3_SPLIT=4" "GEMM4_WNT=2"; do
    env MIPIPE_$v $BB > $O/r9i.log 2>&1 || { tail -3 $O/r9i.log; exit 1; }
    echo "rep $rep $v: mixtral mb256 $(grep -o '"value": [0-9.]*' $O/r9i.log)"
  done
done
