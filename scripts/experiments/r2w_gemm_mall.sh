#!/bin/bash
# GEMM v2 with split-K for narrow shapes; hot (MALL-resident) vs cold single-stream GEMVs; torch (hipBLASLt) f16 GEMM reference
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k gemm > $O/r2w_tests.log 2>&1; rc=$?; tail -2 $O/r2w_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python3 $R/tools/gemv_bench.py --gemm 2 --shapes 70b.gateup,70b.down,70b.qkv,70b.o,8b.gateup,8b.down,8b.qkv --M 512 --iters 6 > $O/gemm2b.log 2>&1 || { tail -5 $O/gemm2b.log; exit 1; }
echo "== gemm v2 split"; grep -oE '"shape": "[^"]*"|"us": [0-9.]+|"TFLOPs": [0-9.]+' $O/gemm2b.log | paste -sd' ' | sed 's/"shape": /\n/g'
for C in 0 1; do
  timeout -k 10 300 python3 $R/tools/gemv_bench.py --copies $C --shapes 8b.qkv,8b.o,8b.gateup,8b.down --M 1 --iters 24 > $O/hot_$C.log 2>&1 || { tail -5 $O/hot_$C.log; exit 1; }
  echo "== M=1 copies=$C"; grep -oE '"shape": "[^"]*"|"us": [0-9.]+' $O/hot_$C.log | paste -sd' ' | sed 's/"shape": /\n/g'
done
timeout -k 10 300 python3 $R/tools/torch_mm_probe.py
