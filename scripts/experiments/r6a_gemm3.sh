#!/bin/bash
# GEMM v3 first light: oracle tests, then v2 vs v3 microbench on the 70B / 8B shapes, then bench.py
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm3_gpu.py > $O/r6a_tests.log 2>&1 || { tail -40 $O/r6a_tests.log; exit 1; }
tail -3 $O/r6a_tests.log
timeout -k 10 300 python -u tools/gemv_bench.py --gemm 2 --M 256 --iters 10 \
  --shapes 70b.qkv,70b.o,70b.gateup,70b.down,8b.gateup,8b.down > $O/r6a_g2.log 2>&1 || { tail -5 $O/r6a_g2.log; exit 1; }
cat $O/r6a_g2.log
timeout -k 10 300 python -u tools/gemv_bench.py --gemm 3 --M 256 --iters 10 \
  --shapes 70b.qkv,70b.o,70b.gateup,70b.down,8b.gateup,8b.down --g3 "0,0,0;256,128,0" > $O/r6a_g3.log 2>&1 || { tail -5 $O/r6a_g3.log; exit 1; }
cat $O/r6a_g3.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/r6a_bench.log 2>&1 || { tail -5 $O/r6a_bench.log; exit 1; }
grep '"value"' $O/r6a_bench.log | cut -c1-200
