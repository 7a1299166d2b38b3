#!/bin/bash
# decode throughput vs micro-batch size (PP=1)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for m in "$@"; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 $m > $O/sweep.log 2>&1 || { tail -5 $O/sweep.log; exit 1; }
  echo "$m: $(grep -o '"value": [0-9.]*, "unit": "tokens/s", "n_gpus": 1, "steps": 20, "warmup": 3, "ms_per_step": [0-9.]*' $O/sweep.log)"
done
