#!/bin/bash
# r12e: full GPU suite on the round-6 build + kernel summaries at mb64 (8B BF16, 70B Q4_K)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r12e_tests.log 2>&1; rc=$?; tail -4 $O/r12e_tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp
prof() { local n=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r12e_$n -- python3 $R/bench.py --steps 30 --warmup 3 --no-secondary "$@" > $O/r12e_$n.log 2>&1 || { tail -3 $O/r12e_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r12e_$n > $O/r12e_prof_$n.txt; rm -rf $O/r12e_$n; echo "== $n $(grep -o '"value": [0-9.]*' $O/r12e_$n.log)"; sed -n '/last 5 decode/,/dispatch order/p' $O/r12e_prof_$n.txt | head -12; }
prof 8b_bf16_mb64 --model llama3-8b --ftype BF16 --mb-size 64
prof 70b_mb64 --model llama3-70b --ftype Q4_K --mb-size 64
prof mixtral_mb256 --model mixtral-8x7b --ftype Q4_K_M --mb-size 256
