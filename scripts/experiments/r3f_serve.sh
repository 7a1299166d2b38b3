#!/bin/bash
# serving benchmark of the orchestrator (8B Q4_K_M, continuous batching): async vs threaded client, 16 / 64 slots
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for cfg in "64 64 async" "64 64 threads" "16 16 async" "64 16 async"; do
  set -- $cfg
  timeout -k 10 400 python3 tools/serve_bench.py --synthetic llama3-8b --ftype Q4_K_M --mb-size $1 --clients $2 --client $3 --requests 4 --modes continuous > $O/serve_$1_$2_$3.log 2>&1 || { tail -20 $O/serve_$1_$2_$3.log; exit 1; }
  tail -1 $O/serve_$1_$2_$3.log
done
