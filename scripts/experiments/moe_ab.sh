#!/bin/bash
# MoE grouped GEMV v2 (workgroup-shared x, MT row groups) vs v1: tests, Mixtral benches, kernel stats
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "moe or engine_matches or spec" > $O/moe_tests.log 2>&1 || { tail -30 $O/moe_tests.log; exit 1; }
tail -1 $O/moe_tests.log
for v in 1 2; do for mb in 64 16 1; do
  MIPIPE_MOE_V=$v timeout -k 10 300 python3 bench.py --model mixtral-8x7b --ftype Q4_K_M --mb-size $mb --steps 20 --warmup 3 > $O/moe_b.log 2>&1 || { tail -5 $O/moe_b.log; exit 1; }
  echo "moe v$v mb$mb: $(grep -o '"value": [0-9.]*' $O/moe_b.log)"
done; done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mx2_prof -o run --output-format csv -- python3 $R/bench.py --model mixtral-8x7b --ftype Q4_K_M --steps 10 --warmup 2 > $O/mx2.log 2>&1 || { tail -5 $O/mx2.log; exit 1; }
python3 $R/tools/prof_summary.py $O/mx2_prof > $O/prof_mixtral_mb64_v2.txt && sed -n "/last 5 decode/,\$p" $O/prof_mixtral_mb64_v2.txt | head -8
