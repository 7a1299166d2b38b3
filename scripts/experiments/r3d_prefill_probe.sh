#!/bin/bash
# gemm2 vs unpack + hipBLASLt at M=2048 and 512
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
for M in 2048 512; do
  timeout -k 10 300 python3 $R/tools/prefill_probe.py --M $M > $O/pp_$M.log 2>&1 || { tail -5 $O/pp_$M.log; exit 1; }
  cat $O/pp_$M.log | grep shape
done
