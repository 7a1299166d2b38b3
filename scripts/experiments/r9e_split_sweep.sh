#!/bin/bash
# r9e: 70B mb256 decode vs the split-K workgroup target (GEMM2_SPLIT_WG: gemm2 / gemm4 split K until
# about this many workgroups; 256 = default), two interleaved reps
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
BB="timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-secondary"
for rep in 1 2; do for w in 256 128 192 384 512; do
  MIPIPE_GEMM2_SPLIT_WG=$w $BB > $O/r9e_$w.log 2>&1 || { tail -3 $O/r9e_$w.log; exit 1; }
  echo "rep $rep GEMM2_SPLIT_WG=$w: 70b mb256 $(grep -o '"value": [0-9.]*' $O/r9e_$w.log)"
done; done
