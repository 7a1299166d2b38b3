#!/bin/bash
# probe: A fragments from registers instead of LDS reads (timing only) vs the production GEMV at M=64
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
for L in libmipipe.so lib_nolds.so; do
  MIPIPE_LIB=$L timeout -k 10 200 python3 $R/tools/gemv_bench.py --shapes 70b.gateup,70b.down,70b.qkv,70b.o --M 64 --iters 12 > $O/nl_$L.log 2>&1 || { tail -5 $O/nl_$L.log; exit 1; }
  echo "== $L: $(grep -oE '"shape": "[^"]*"|"us": [0-9.]+' $O/nl_$L.log | paste -sd' ' | sed 's/"shape": //g')"
done
