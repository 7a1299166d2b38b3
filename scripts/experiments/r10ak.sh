#!/bin/bash
# r10ak: 70B mb256 with the 4-wave gate/up tiles: non-temporal weight DMA (GEMM4_WNT auto = on for one row block) vs plain
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
for rep in 1 2 3; do
  for v in 0 2; do
    MIPIPE_GEMM4_WNT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-secondary > $O/r10ak.log 2>&1 || { tail -5 $O/r10ak.log; exit 1; }
    echo "rep $rep 70b mb256 GEMM4_WNT=$v $(grep -o '"value": [0-9.]*' $O/r10ak.log)"
  done
done
