#!/bin/bash
# r11c: (1) the engine tests around the new qkv append epilogue; (2) 8B Q4_K_M single stream per-kernel times:
# ATTN_PRE 0 / 1, gemvs residual prefetch (GEMVS_RPF 0 / 1), 8-wave attention, and the gemvs timing probes
# (probe library, GEMVS_PROBE bits: 1 no dequant/MFMA, 2 no x prologue, 4 plain epilogue store)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_hybrid_gpu.py -k "qkv_append or matches_reference or fused_decode or fused_norm or graph_equals or local_link or pipeline_emulation or hybrid" > $O/r11c_tests.log 2>&1; rc=$?; tail -5 $O/r11c_tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp
prof() { local n=$1; shift; timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r11c_$n -- python3 $R/bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 30 --warmup 3 --no-secondary > $O/r11c_$n.log 2>&1 || { tail -3 $O/r11c_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r11c_$n > $O/r11c_prof_$n.txt; rm -rf $O/r11c_$n; echo "== $n $(grep -o '"value": [0-9.]*' $O/r11c_$n.log)"; sed -n '/last 5 decode/,/dispatch order/p' $O/r11c_prof_$n.txt | head -9; }
prof new
MIPIPE_ATTN_PRE=0 prof pre0
MIPIPE_GEMVS_RPF=0 prof rpf0
MIPIPE_ATTN_NW8_MAXWG=64 prof nw8
