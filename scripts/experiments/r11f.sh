#!/bin/bash
# r11f: the single-row v_dot2 GEMV form (GEMVS_DOT): oracle tests, engine tests, 8B Q4_K_M mb1 profiles DOT 1 / 0
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemvs_gpu.py tests/test_engine_gpu.py -k "gemvs or matches_reference or qkv_append or fused_norm" > $O/r11f_tests.log 2>&1; rc=$?; tail -4 $O/r11f_tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp
prof() { local n=$1; shift; timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r11f_$n -- python3 $R/bench.py --steps 30 --warmup 3 --no-secondary "$@" > $O/r11f_$n.log 2>&1 || { tail -3 $O/r11f_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r11f_$n > $O/r11f_prof_$n.txt; rm -rf $O/r11f_$n; echo "== $n $(grep -o '"value": [0-9.]*' $O/r11f_$n.log)"; sed -n '/last 5 decode/,/dispatch order/p' $O/r11f_prof_$n.txt | head -9; }
prof dot1 --model llama3-8b --ftype Q4_K_M --mb-size 1
MIPIPE_GEMVS_DOT=0 prof dot0 --model llama3-8b --ftype Q4_K_M --mb-size 1
prof 70b_dot1 --mb-size 1
