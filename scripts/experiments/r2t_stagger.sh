#!/bin/bash
# staggered SIMD partners in the M > 48 GEMV: kernel tests, micro-bench and engine A/B per switch value
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py > $O/r2t_tests.log 2>&1; rc=$?; tail -2 $O/r2t_tests.log; [ $rc = 0 ] || exit 1
for S in 0 1 2 3; do
  MIPIPE_GEMV_STAGGER=$S timeout -k 10 200 python3 $R/tools/gemv_bench.py --shapes 70b.gateup,70b.down,70b.qkv,70b.o --M 64 --iters 12 > $O/stg_$S.log 2>&1 || { tail -5 $O/stg_$S.log; exit 1; }
  echo "== stagger $S: $(grep -oE '"shape": "[^"]*"|"us": [0-9.]+' $O/stg_$S.log | paste -sd' ' | sed 's/"shape": //g')"
done
for S in 0 3 2 0 3 2; do
  MIPIPE_GEMV_STAGGER=$S timeout -k 10 200 python3 $R/bench.py --steps 20 --warmup 5 > $O/stgb_$S.log 2>&1 || { tail -5 $O/stgb_$S.log; exit 1; }
  echo "bench stagger $S: $(grep -o '"value": [0-9.]*' $O/stgb_$S.log)"
done
