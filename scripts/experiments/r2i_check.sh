#!/bin/bash
# full GPU suite + single-stream A/B (deferred norm on/off) + headline
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r2i_tests.log 2>&1 || { tail -40 $O/r2i_tests.log; exit 1; }
tail -2 $O/r2i_tests.log
for v in on off; do
  timeout -k 10 200 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 50 --set fused_norm=$([ $v = on ] && echo true || echo false) > $O/r2i_bench8b_$v.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --mb-size 1 --steps 20 --set fused_norm=$([ $v = on ] && echo true || echo false) > $O/r2i_bench70b_mb1_$v.log 2>&1 || exit 1
done
timeout -k 10 200 python bench.py > $O/r2i_bench70b_mb64.log 2>&1 || exit 1
