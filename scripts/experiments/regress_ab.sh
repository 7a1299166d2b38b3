#!/bin/bash
# same-box A/B: current tree vs the build of an earlier commit in old_ab/ (70B mb64 headline)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
for rep in 1 2; do
  cd $R && timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > $O/ra_new.log 2>&1 || { tail -5 $O/ra_new.log; exit 1; }
  echo "new: $(grep -o '"value": [0-9.]*' $O/ra_new.log)"
  cd $R/old_ab && timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > $O/ra_old.log 2>&1 || { tail -5 $O/ra_old.log; exit 1; }
  echo "old: $(grep -o '"value": [0-9.]*' $O/ra_old.log)"
done
