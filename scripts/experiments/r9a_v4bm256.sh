#!/bin/bash
# r9a: 70B mb256 decode with gemm4 on the split-K shapes at 256-row tiles (more K splits, half the
# dequant per MFMA of the 128-row tiles) vs the default (gemm2 there) vs gemm4 at the auto 128 rows
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
BB="timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-secondary"
for rep in 1 2; do
  $BB > $O/r9a_def.log 2>&1 || { tail -3 $O/r9a_def.log; exit 1; }
  $BB --set prefill_gemm_v=4 > $O/r9a_v4.log 2>&1 || { tail -3 $O/r9a_v4.log; exit 1; }
  MIPIPE_GEMM3_BM=256 $BB --set prefill_gemm_v=4 > $O/r9a_v4bm.log 2>&1 || { tail -3 $O/r9a_v4bm.log; exit 1; }
  echo "rep $rep: default $(grep -o '"value": [0-9.]*' $O/r9a_def.log) | v4 $(grep -o '"value": [0-9.]*' $O/r9a_v4.log) | v4 bm256 $(grep -o '"value": [0-9.]*' $O/r9a_v4bm.log)"
done
