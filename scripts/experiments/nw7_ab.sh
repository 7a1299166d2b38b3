#!/bin/bash
# 7- vs 8-wave workgroups for the two-tiles-per-wave gate/up GEMV: correctness, micro-bench, engine bench
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
MIPIPE_GEMV2_TW=2 MIPIPE_GEMV2_TW2_NW=7 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k gemv > $O/nw7_tests.log 2>&1 || { tail -30 $O/nw7_tests.log; exit 1; }
tail -1 $O/nw7_tests.log
for nw in 8 7; do
  MIPIPE_GEMV2_TW2_NW=$nw timeout -k 10 200 python3 tools/gemv_bench.py --shapes 70b.gateup --M 33,48,64 --tpw 1 > $O/nw7_$nw.log 2>&1 || { tail -5 $O/nw7_$nw.log; exit 1; }
  echo "NW=$nw: $(grep -o '"M": [0-9]*\|"us": [0-9.]*' $O/nw7_$nw.log | paste - - | tr '\n' ' ')"
done
for rep in 1 2; do for nw in 8 0; do
  MIPIPE_GEMV2_TW2_NW=$nw timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > $O/nw7_b.log 2>&1 || { tail -5 $O/nw7_b.log; exit 1; }
  echo "bench TW2_NW=$nw: $(grep -o '"value": [0-9.]*' $O/nw7_b.log)"
done; done
