#!/bin/bash
# A/B the gemv2 ring depths (weights NSW x NSX for M > 32) on the 70B Q4_K decode shapes
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for L in libmipipe_w2x2.so libmipipe_w3x2.so libmipipe_w4x2.so libmipipe_w3x3.so libmipipe_w4x3.so; do
  echo "== $L"
  MIPIPE_LIB=$L timeout -k 10 200 python3 tools/gemv_bench.py --shapes 70b.gateup,70b.down,70b.qkv,70b.o --M 48,64 --tpw 1 > $O/probe_$L.log 2>&1 || { tail -5 $O/probe_$L.log; exit 1; }
  grep -o '"shape": "[^"]*".*"M": [0-9]*\|"us": [0-9.]*' $O/probe_$L.log | paste - - | awk '{print $2, $8, $10}'
done
