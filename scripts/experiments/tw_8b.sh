#!/bin/bash
# 8B / 70B mb64 with the grid-size rule for two tiles per wave (auto) vs forced TW=1 / TW=2
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for m in "llama3-8b Q4_K_M" "llama3-70b Q4_K"; do
  set -- $m
  for tw in 0 1 2; do
    MIPIPE_GEMV2_TW=$tw timeout -k 10 300 python3 bench.py --model $1 --ftype $2 --steps 20 --warmup 3 > $O/tw8_$1_$tw.log 2>&1 || { tail -5 $O/tw8_$1_$tw.log; exit 1; }
    echo "$1 TW=$tw: $(grep -o '"value": [0-9.]*' $O/tw8_$1_$tw.log)"
  done
done
