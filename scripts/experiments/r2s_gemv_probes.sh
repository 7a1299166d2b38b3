#!/bin/bash
# M=64 GEMV cost probes (timing only for nobar / nodeq / mfma4) + NSLOT=3 engine A/B
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
for L in libmipipe.so lib_ns3.so lib_nobar.so lib_nodeq.so lib_mfma4.so; do
  MIPIPE_LIB=$L timeout -k 10 200 python3 $R/tools/gemv_bench.py --shapes 70b.gateup,70b.down,70b.qkv,70b.o --M 64 --iters 12 > $O/gp_$L.log 2>&1 || { tail -5 $O/gp_$L.log; exit 1; }
  echo "== $L"; grep -oE '"shape": "[^"]*"|"us": [0-9.]+' $O/gp_$L.log | paste -sd' ' | sed 's/"shape"/\n/g'
done
for L in libmipipe.so lib_ns3.so libmipipe.so lib_ns3.so; do
  MIPIPE_LIB=$L timeout -k 10 200 python3 $R/bench.py --steps 20 --warmup 5 > $O/gpb_$L.log 2>&1 || { tail -5 $O/gpb_$L.log; exit 1; }
  echo "bench $L: $(grep -o '"value": [0-9.]*' $O/gpb_$L.log)"
done
