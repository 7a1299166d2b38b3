#!/bin/bash
# producer-tail RMSNorm: GPU tests, then single-stream benches on/off
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/r3a_tests.log 2>&1; rc=$?; tail -3 $O/r3a_tests.log; [ $rc = 0 ] || exit 1
for T in true false true false; do
  timeout -k 10 300 python3 bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 50 --set tail_norm=$T > $O/r3a_8b_$T.log 2>&1 || { tail -5 $O/r3a_8b_$T.log; exit 1; }
  echo "8B mb1 tail_norm=$T $(grep -o '"value": [0-9.]*' $O/r3a_8b_$T.log)"
done
for T in true false; do
  timeout -k 10 300 python3 bench.py --mb-size 1 --set tail_norm=$T > $O/r3a_70b_$T.log 2>&1 || { tail -5 $O/r3a_70b_$T.log; exit 1; }
  echo "70B mb1 tail_norm=$T $(grep -o '"value": [0-9.]*' $O/r3a_70b_$T.log)"
done
bash $R/scripts/experiments/prof_mb.sh t8b --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 30
