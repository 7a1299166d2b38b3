#!/bin/bash
# r12g: gemm2 retired (full GPU suite), one-round residual GEMVs with 4 super-blocks in flight per wave; 8B / 70B mb1 profiles
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r12g_tests.log 2>&1; rc=$?; tail -4 $O/r12g_tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp
prof() { local n=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r12g_$n -- python3 $R/bench.py --steps 30 --warmup 3 --no-secondary "$@" > $O/r12g_$n.log 2>&1 || { tail -3 $O/r12g_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r12g_$n > $O/r12g_prof_$n.txt; rm -rf $O/r12g_$n; echo "== $n $(grep -o '"value": [0-9.]*' $O/r12g_$n.log)"; sed -n '/last 5 decode/,/dispatch order/p' $O/r12g_prof_$n.txt | head -12; }
prof 8b_mb1 --model llama3-8b --ftype Q4_K_M --mb-size 1
prof 70b_mb1 --model llama3-70b --ftype Q4_K --mb-size 1
