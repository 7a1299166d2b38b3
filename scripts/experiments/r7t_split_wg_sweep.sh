#!/bin/bash
# gemm2 split-K workgroup target with partial stores (round 2's sweep was with atomics: 256 best)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for wg in 256 384 512 192 256; do
  timeout -k 10 300 env MIPIPE_GEMM2_SPLIT_WG=$wg python bench.py --steps 15 --warmup 3 --no-secondary > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "70b mb256 split_wg=$wg $(grep -o '"value": [0-9.]*' $O/b.log)"
done
for wg in 256 512; do
  timeout -k 10 300 env MIPIPE_GEMM2_SPLIT_WG=$wg python bench.py --model llama3-8b --ftype Q4_K_M --steps 15 --warmup 3 --no-secondary > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "8b mb256 split_wg=$wg $(grep -o '"value": [0-9.]*' $O/b.log)"
done
