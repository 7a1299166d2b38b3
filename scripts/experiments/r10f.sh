#!/bin/bash
# r10f: MoE weight DMA non-temporal (auto) vs plain in the engine (Mixtral mb256 / mb64), then the GPU suite
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
for rep in 1 2; do
  for w in 0 2; do
    MIPIPE_GEMM4_WNT=$w timeout -k 10 300 python bench.py --model mixtral-8x7b --ftype Q4_K_M --steps 10 --warmup 3 --no-secondary > $O/r10f_mx$w.log 2>&1 || { tail -5 $O/r10f_mx$w.log; exit 1; }
    echo "rep $rep mixtral mb256 GEMM4_WNT=$w $(grep -o '"value": [0-9.]*' $O/r10f_mx$w.log)"
  done
done
for w in 0 2; do
  MIPIPE_GEMM4_WNT=$w timeout -k 10 300 python bench.py --model mixtral-8x7b --ftype Q4_K_M --mb-size 64 --steps 10 --warmup 3 --no-secondary > $O/r10f_mx64_$w.log 2>&1 || exit 1
  echo "mixtral mb64 GEMM4_WNT=$w $(grep -o '"value": [0-9.]*' $O/r10f_mx64_$w.log)"
done
exit 0
