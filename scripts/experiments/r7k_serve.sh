#!/bin/bash
# serving benchmark of the orchestrator after the round-3 changes: 8B Q4_K_M, continuous batching, 64 and
# 256 slots (the wide-micro-batch GEMM path with admits into rows >= 64)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for cfg in "64 64" "256 128" "256 256"; do
  set -- $cfg
  timeout -k 10 400 python3 tools/serve_bench.py --synthetic llama3-8b --ftype Q4_K_M --mb-size $1 --clients $2 --client async --requests 4 --modes continuous > $O/serve_$1_$2.log 2>&1 || { tail -20 $O/serve_$1_$2.log; exit 1; }
  tail -1 $O/serve_$1_$2.log
done
