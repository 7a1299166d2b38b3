#!/bin/bash
# gemm2 split-K workgroup target for the accumulate shapes (qkv / o / down) at the headline mb256
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for w in 256 128 192 384 512 256; do
  MIPIPE_GEMM2_SPLIT_WG=$w timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/r5n.log 2>&1 || { tail -5 $O/r5n.log; exit 1; }
  echo "split_wg=$w 70b mb256 $(grep -o '"value": [0-9.]*' $O/r5n.log)"
done
