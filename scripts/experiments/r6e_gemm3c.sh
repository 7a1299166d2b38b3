#!/bin/bash
# GEMM v3c (cross-stage MFMA stream, weights issued 3 stages ahead) vs gemm2: tests, shapes, bench A/B
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm3_gpu.py tests/test_kernels_gpu.py > $O/r6e_tests.log 2>&1 || { tail -40 $O/r6e_tests.log; exit 1; }
tail -2 $O/r6e_tests.log
SH=70b.qkv,70b.o,70b.gateup,70b.down,8b.gateup,8b.down
timeout -k 10 300 python -u tools/gemv_bench.py --gemm 3 --M 256 --iters 20 --shapes $SH --g3 "0,0,0;256,128,0" \
  > $O/r6e_g3.log 2>&1 || { tail -5 $O/r6e_g3.log; exit 1; }
timeout -k 10 300 python -u tools/gemv_bench.py --gemm 2 --M 256 --iters 20 --shapes $SH \
  > $O/r6e_g2.log 2>&1 || { tail -5 $O/r6e_g2.log; exit 1; }
grep shape $O/r6e_g3.log $O/r6e_g2.log | cut -c1-200
timeout -k 10 300 python -u tools/gemv_bench.py --gemm 3 --M 256 --iters 20 --shapes 70b.gateup \
  --knob GEMM3_PROBE=0,1,2,3,4,6 > $O/r6e_probes.log 2>&1 || { tail -5 $O/r6e_probes.log; exit 1; }
grep shape $O/r6e_probes.log | cut -c1-200
for v in 3 2 3; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-secondary --set prefill_gemm_v=$v > $O/r6e_bench_v$v.log 2>&1 \
    || { tail -5 $O/r6e_bench_v$v.log; exit 1; }
  echo "v$v $(grep -o '"value": [0-9.]*' $O/r6e_bench_v$v.log)"
done
