#!/bin/bash
# gemv2 TW=2 software-pipelined step vs TW=1: correctness + 70B decode shapes at M=48/64 + engine bench
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for tw in 2 1; do
MIPIPE_GEMV2_TW=$tw timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k gemv > $O/tw_tests.log 2>&1 || { tail -30 $O/tw_tests.log; exit 1; }
tail -1 $O/tw_tests.log
done
for tw in 1 2; do
  echo "== TW=$tw"
  MIPIPE_GEMV2_TW=$tw timeout -k 10 200 python3 tools/gemv_bench.py --shapes 70b.gateup,70b.down,70b.qkv,70b.o --M 48,64 --tpw 1 --splits 2,4,8 > $O/tw2_$tw.log 2>&1 || { tail -5 $O/tw2_$tw.log; exit 1; }
  python3 -c "
import json,sys
for l in open('$O/tw2_$tw.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], d['M'], d['nsplit'], d['us'])" | paste - - - - 
done
for tw in 0 2 1; do
  MIPIPE_GEMV2_TW=$tw timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > $O/tw_bench_$tw.log 2>&1 || { tail -5 $O/tw_bench_$tw.log; exit 1; }
  echo "bench TW=$tw: $(grep -o '"value": [0-9.]*' $O/tw_bench_$tw.log)"
done
