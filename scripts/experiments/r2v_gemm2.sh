#!/bin/bash
# prompt GEMM v2 (128 x 256 workgroup tiles): oracle tests, micro-bench vs the 64x64 GEMM, then single-stream profiles
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k gemm > $O/r2v_tests.log 2>&1; rc=$?; tail -2 $O/r2v_tests.log; [ $rc = 0 ] || exit 1
for G in 1 2; do
  timeout -k 10 300 python3 $R/tools/gemv_bench.py --gemm $G --shapes 70b.gateup,70b.down,70b.qkv,70b.o,8b.gateup,8b.down,8b.qkv --M 512 --iters 6 > $O/gemm_$G.log 2>&1 || { tail -5 $O/gemm_$G.log; exit 1; }
  echo "== gemm v$G"; grep -oE '"shape": "[^"]*"|"us": [0-9.]+|"TFLOPs": [0-9.]+' $O/gemm_$G.log | paste -sd' ' | sed 's/"shape": /\n/g'
done
bash $R/scripts/experiments/r2u_prof_mb1.sh
