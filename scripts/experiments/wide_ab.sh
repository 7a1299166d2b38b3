#!/bin/bash
# A/B of the wide (3-4 row group) GEMV variants: MIPIPE_GEMV_WIDE = 0 / 1 / 2
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for v in 0 1 2; do
  echo "== variant $v"
  MIPIPE_GEMV_WIDE=$v timeout -k 10 200 python3 tools/gemv_bench.py --shapes 70b.qkv,70b.o,70b.gateup,70b.down --M 48,64 --tpw 1 > $O/wide_$v.log 2>&1 || { tail -5 $O/wide_$v.log; exit 1; }
  grep -o '"shape": "[^"]*".*"M": [0-9]*\|"us": [0-9.]*' $O/wide_$v.log | paste - - | awk '{print $2, $8, $10}'
  MIPIPE_GEMV_WIDE=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 > $O/wide_b$v.log 2>&1 || { tail -5 $O/wide_b$v.log; exit 1; }
  grep -o '"value": [0-9.]*' $O/wide_b$v.log
done
