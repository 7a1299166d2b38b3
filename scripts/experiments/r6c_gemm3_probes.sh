#!/bin/bash
# GEMM v3 timing probes on 70B gate/up M=256 (Q4_K, 256x256): full / no MFMA / no dequant / neither / no staging
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u tools/gemv_bench.py --gemm 3 --M 256 --iters 10 --shapes 70b.gateup \
  --knob GEMM3_PROBE=0,1,2,3,4,6,0 > $O/r6c_probes.log 2>&1 || { tail -5 $O/r6c_probes.log; exit 1; }
grep shape $O/r6c_probes.log
