#!/bin/bash
# 16-wave workgroups (x staged once per 16 tiles) for the M=64 one-tile GEMVs vs 8-wave, split sweep
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "saturates or swiglu" > $O/r3c_tests.log 2>&1; rc=$?; tail -2 $O/r3c_tests.log; [ $rc = 0 ] || exit 1; cd /tmp
for NW in 8 16; do
  MIPIPE_LIB=lib_nw16.so MIPIPE_GEMV_NW=$NW timeout -k 10 300 python3 $R/tools/gemv_bench.py --shapes 70b.qkv,70b.o,70b.down --M 64 --splits 2,4,8 --iters 12 > $O/nw_$NW.log 2>&1 || { tail -5 $O/nw_$NW.log; exit 1; }
  MIPIPE_LIB=lib_nw16.so MIPIPE_GEMV_NW=$NW timeout -k 10 300 python3 $R/tools/gemv_bench.py --shapes 70b.gateup --M 64 --iters 12 >> $O/nw_$NW.log 2>&1 || { tail -5 $O/nw_$NW.log; exit 1; }
  echo "== NW=$NW"; grep -oE '"shape": "[^"]*"|"nsplit": [0-9]+|"us": [0-9.]+' $O/nw_$NW.log | paste -sd' ' | sed 's/"shape": /\n/g'
done
for NW in 8 16 8 16; do
  MIPIPE_LIB=lib_nw16.so MIPIPE_GEMV_NW=$NW timeout -k 10 200 python3 $R/bench.py > $O/nwb_$NW.log 2>&1 || { tail -5 $O/nwb_$NW.log; exit 1; }
  echo "bench NW=$NW $(grep -o '"value": [0-9.]*' $O/nwb_$NW.log)"
done
