#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for S in 32 64 128; do
  MIPIPE_GEMVS_S=$S timeout -k 10 300 python bench.py --mb-size 1 --steps 20 --warmup 3 > $O/r5h_$S.log 2>&1 || { tail -5 $O/r5h_$S.log; exit 1; }
  echo "S=$S 70b mb1 $(grep -o '"value": [0-9.]*' $O/r5h_$S.log)"
done
timeout -k 10 300 python bench.py --mb-size 1 --steps 20 --warmup 3 --set small_gemv=false > $O/r5h_old.log 2>&1 || { tail -5 $O/r5h_old.log; exit 1; }
echo "gemv2 path 70b mb1 $(grep -o '"value": [0-9.]*' $O/r5h_old.log)"
for S in 16 32 64; do
  MIPIPE_GEMVS_S=$S timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 30 --warmup 3 > $O/r5h_8b_$S.log 2>&1 || { tail -5 $O/r5h_8b_$S.log; exit 1; }
  echo "S=$S 8b mb1 $(grep -o '"value": [0-9.]*' $O/r5h_8b_$S.log)"
done
