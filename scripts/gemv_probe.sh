#!/bin/bash
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/probe; mkdir -p $O; cd $R
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -p no:cacheprovider -k "gemm or gemv" > $O/kt.log 2>&1; rc=$?; tail -3 $O/kt.log
[ $rc -ne 0 ] && exit $rc
for PR in 0 3 4 5; do for XR in 0 1; do
  MIPIPE_GEMV_XR=$XR timeout -k 10 200 python tools/gemv_bench.py --shapes 70b.gateup,70b.down --types Q4_K --M 1,16 --tpw 1,2,4 --probe $PR > $O/p${PR}_xr$XR.log 2>&1 || { tail -3 $O/p${PR}_xr$XR.log; exit 1; }
done; done
cd $O; for f in p*_xr*.log; do echo "== $f"; grep shape $f | sed -E 's/.*"shape": "([^"]+)".*"M": ([0-9]+), "tpw": ([0-9]), "nsplit": ([0-9]+), "us": ([0-9.]+).*/\1 M\2 t\3 s\4 \5/' | paste -sd' ' ; done
