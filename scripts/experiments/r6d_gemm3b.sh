#!/bin/bash
# GEMM v3b (wave-owned columns, 3-deep all-LDS-DMA pipeline): oracle tests, probes, v2 vs v3 shapes, bench.py
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm3_gpu.py > $O/r6d_tests.log 2>&1 || { tail -40 $O/r6d_tests.log; exit 1; }
tail -2 $O/r6d_tests.log
timeout -k 10 300 python -u tools/gemv_bench.py --gemm 3 --M 256 --iters 10 --shapes 70b.gateup \
  --knob GEMM3_PROBE=0,1,2,3,4,6,0 > $O/r6d_probes.log 2>&1 || { tail -5 $O/r6d_probes.log; exit 1; }
grep shape $O/r6d_probes.log | cut -c1-200
timeout -k 10 300 python -u tools/gemv_bench.py --gemm 3 --M 256 --iters 10 \
  --shapes 70b.qkv,70b.o,70b.gateup,70b.down,8b.gateup,8b.down --g3 "0,0,0;256,128,0" > $O/r6d_g3.log 2>&1 || { tail -5 $O/r6d_g3.log; exit 1; }
grep shape $O/r6d_g3.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-secondary > $O/r6d_bench.log 2>&1 || { tail -5 $O/r6d_bench.log; exit 1; }
grep '"value"' $O/r6d_bench.log | cut -c1-250
