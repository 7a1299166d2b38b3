#!/bin/bash
# r10am: kernel summaries of the final round-5 build: Mixtral 8x7B Q4_K_M mb256, Llama-3-8B Q4_K_M single stream,
# Llama-3-70B Q4_K mb64
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
prof() { local n=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r10am_$n -- python3 $R/bench.py --steps 10 --warmup 2 --no-secondary "$@" > $O/r10am_$n.log 2>&1 || { tail -3 $O/r10am_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r10am_$n > $O/r10am_prof_$n.txt; rm -rf $O/r10am_$n; echo "== $n $(grep -o '"value": [0-9.]*' $O/r10am_$n.log)"; sed -n '/last 5 decode/,/dispatch order/p' $O/r10am_prof_$n.txt | head -10; }
prof mixtral_mb256 --model mixtral-8x7b --ftype Q4_K_M
prof 8b_mb1 --model llama3-8b --ftype Q4_K_M --mb-size 1
prof 70b_mb64 --mb-size 64
