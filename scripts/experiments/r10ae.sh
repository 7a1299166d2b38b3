#!/bin/bash
# r10ae: 70B mb64 -- split-K atomics (default) vs per-split partial stores + a fixed-order reduction (deterministic mode)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
for rep in 1 2; do
  for d in false true; do
    timeout -k 10 200 python bench.py --mb-size 64 --steps 8 --warmup 2 --no-secondary --set deterministic=$d > $O/r10ae.log 2>&1 || { tail -3 $O/r10ae.log; exit 1; }
    echo "rep $rep 70b mb64 deterministic=$d $(grep -o '"value": [0-9.]*' $O/r10ae.log)"
  done
done
