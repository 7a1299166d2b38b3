#!/bin/bash
# GEMV sweep: intra-workgroup split-K (MIPIPE_GEMV_KS) x fast dequant experiment; then kernel tests with KS=2,4
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/ks; mkdir -p $O; cd $R
for KS in 2 4; do
  MIPIPE_GEMV_KS=$KS timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -p no:cacheprovider -k gemv > $O/kt$KS.log 2>&1; rc=$?; tail -1 $O/kt$KS.log
  [ $rc -ne 0 ] && exit $rc
done
for KS in 1 2 4; do for XR in 0 1; do
  MIPIPE_GEMV_KS=$KS MIPIPE_GEMV_XR=$XR timeout -k 10 200 python tools/gemv_bench.py --shapes 70b.qkv,70b.o,70b.gateup,70b.down,70b.head --types Q4_K --M 1,16 --tpw 1,2,4 > $O/ks${KS}_xr$XR.log 2>&1 || { tail -3 $O/ks${KS}_xr$XR.log; exit 1; }
done; done
cd $O; for f in ks*_xr*.log; do echo "== $f"; grep shape $f | sed -E 's/.*"shape": "([^"]+)".*"M": ([0-9]+), "tpw": ([0-9]), "nsplit": ([0-9]+), "us": ([0-9.]+).*/\1 M\2 t\3 s\4 \5/' | paste -sd' ' ; done
