#!/bin/bash
# gemv2 tiles-per-wave A/B (MIPIPE_GEMV2_TW x MIPIPE_GEMV_NW) at M = 48/64: correctness, micro-bench, engine bench
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
MIPIPE_GEMV2_TW=2 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k gemv > $O/tw_tests.log 2>&1 || { tail -30 $O/tw_tests.log; exit 1; }
tail -2 $O/tw_tests.log
for cfg in "1 8" "2 8" "2 4"; do
  set -- $cfg
  echo "== TW=$1 NW=$2"
  MIPIPE_GEMV2_TW=$1 MIPIPE_GEMV_NW=$2 timeout -k 10 200 python3 tools/gemv_bench.py --shapes 70b.gateup,70b.down,70b.qkv,70b.o --M 48,64 --tpw 1 --splits 2,4,8,16 > $O/tw_$1_$2.log 2>&1 || { tail -5 $O/tw_$1_$2.log; exit 1; }
  python3 -c "
import json,sys
for l in open('$O/tw_$1_$2.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], d['M'], d['nsplit'], d['us'])" | paste - - - - 
done
for tw in 1 2; do
  MIPIPE_GEMV2_TW=$tw timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > $O/tw_bench_$tw.log 2>&1 || { tail -5 $O/tw_bench_$tw.log; exit 1; }
  echo "bench TW=$tw: $(grep -o '"value": [0-9.]*' $O/tw_bench_$tw.log)"
done
