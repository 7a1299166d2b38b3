#!/bin/bash
# r10u: GEMM4_TW4=1 (4 waves x 64 columns on the 256-row gate/up tiles only) vs 0, engine A/B alternated: 70B / 8B mb256
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
for rep in 1 2 3; do
  for v in 0 1; do
    MIPIPE_GEMM4_TW4=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-secondary > $O/r10u_70b_$v.log 2>&1 || { tail -5 $O/r10u_70b_$v.log; exit 1; }
    echo "rep $rep 70b mb256 GEMM4_TW4=$v $(grep -o '"value": [0-9.]*' $O/r10u_70b_$v.log)"
  done
done
for v in 0 1; do
  MIPIPE_GEMM4_TW4=$v timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --steps 10 --warmup 3 --no-secondary > $O/r10u_8b_$v.log 2>&1 || { tail -5 $O/r10u_8b_$v.log; exit 1; }
  echo "8b mb256 GEMM4_TW4=$v $(grep -o '"value": [0-9.]*' $O/r10u_8b_$v.log)"
done
