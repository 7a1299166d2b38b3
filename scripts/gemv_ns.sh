#!/bin/bash
# GEMV sweep over super-blocks in flight (MIPIPE_GEMV_NSLOT) x fast-dequant experiment (MIPIPE_GEMV_XR)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/ns; mkdir -p $O; cd $R
for NS in 0 4 3 8; do for XR in 0 1; do
  MIPIPE_GEMV_NSLOT=$NS MIPIPE_GEMV_XR=$XR timeout -k 10 200 python tools/gemv_bench.py --shapes 70b.qkv,70b.gateup,70b.down --types Q4_K --M 1,16 --tpw 1,2,4 > $O/ns${NS}_xr$XR.log 2>&1 || { tail -3 $O/ns${NS}_xr$XR.log; exit 1; }
done; done
cd $O; for f in ns*_xr*.log; do echo "== $f"; grep shape $f | sed -E 's/.*"shape": "([^"]+)".*"M": ([0-9]+), "tpw": ([0-9]), "nsplit": ([0-9]+), "us": ([0-9.]+).*/\1 M\2 tpw\3 s\4 \5/' | paste -sd' ' ; done
