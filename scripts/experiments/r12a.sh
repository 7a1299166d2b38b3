#!/bin/bash
# r12a: pipeline overhead with the posted-queue LocalLink -- 8B BF16 mb64 PP=1 vs PP=4 on one GPU (same device),
# 70B Q4_K mb256 PP=1 vs PP=8 (same device); span traces of the PP runs (5 rounds after the timed region)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 300 python3 -u $R/bench.py --no-secondary "$@" > $O/r12a_$n.log 2>&1 || { tail -5 $O/r12a_$n.log; exit 1; }
  echo "== $n $(grep -o '"value": [0-9.]*' $O/r12a_$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r12a_$n.log)"; }
run 8b_pp1 --model llama3-8b --ftype BF16 --mb-size 64 --trace $O/r12a_8b_pp1.trace.json
run 8b_pp4 --model llama3-8b --ftype BF16 --mb-size 64 --gpus 4 --same-device --trace $O/r12a_8b_pp4.trace.json
run 70b_pp1 --model llama3-70b --ftype Q4_K --mb-size 256
run 70b_pp8 --model llama3-70b --ftype Q4_K --mb-size 256 --gpus 8 --same-device --trace $O/r12a_70b_pp8.trace.json
