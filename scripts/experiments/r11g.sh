#!/bin/bash
# r11g: fused attention + o-projection (attn_o, now on the pre-appended q/K/V) vs two kernels, 8B Q4_K_M mb1;
# Q6_K down back on the MFMA form
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py -k "attention_o or qkv_append or matches_reference" > $O/r11g_tests.log 2>&1; rc=$?; tail -4 $O/r11g_tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp
prof() { local n=$1; shift; timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r11g_$n -- python3 $R/bench.py --steps 30 --warmup 3 --no-secondary "$@" > $O/r11g_$n.log 2>&1 || { tail -3 $O/r11g_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r11g_$n > $O/r11g_prof_$n.txt; rm -rf $O/r11g_$n; echo "== $n $(grep -o '"value": [0-9.]*' $O/r11g_$n.log)"; sed -n '/last 5 decode/,/dispatch order/p' $O/r11g_prof_$n.txt | head -10; }
prof two --model llama3-8b --ftype Q4_K_M --mb-size 1
prof fused --model llama3-8b --ftype Q4_K_M --mb-size 1 --set attn_o_max_ctx=4096
