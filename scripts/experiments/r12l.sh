#!/bin/bash
# r12l: 7-wave 128-row gemm4 tiles at two workgroups per CU (GEMM4_TW4 7: gate/up, 8: every dense shape);
# MoE down split over K (GEMM3_SPLIT) with the 96-row tiles
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm4_gpu.py -k "four_wave" > $O/r12l_tests.log 2>&1; rc=$?; tail -3 $O/r12l_tests.log; [ $rc -ne 0 ] && exit $rc
run() { local n=$1 e="$2"; shift 2; timeout -k 10 300 env $e python3 -u $R/bench.py --no-secondary "$@" > $O/r12l_$n.log 2>&1 || { tail -5 $O/r12l_$n.log; exit 1; }
  echo "== $n $(grep -o '"value": [0-9.]*' $O/r12l_$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r12l_$n.log)"; }
run 70b_tw1 "MIPIPE_GEMM4_TW4=1"
run 70b_tw7 "MIPIPE_GEMM4_TW4=7"
run 70b_tw8 "MIPIPE_GEMM4_TW4=8"
run 70b_tw1b "MIPIPE_GEMM4_TW4=1"
run 70b_tw7b "MIPIPE_GEMM4_TW4=7"
run 8b_tw1 "MIPIPE_GEMM4_TW4=1" --model llama3-8b --ftype Q4_K_M --mb-size 256
run 8b_tw7 "MIPIPE_GEMM4_TW4=7" --model llama3-8b --ftype Q4_K_M --mb-size 256
for s in 0 2 4; do run mix_split$s "MIPIPE_GEMM3_SPLIT=$s" --model mixtral-8x7b --ftype Q4_K_M --mb-size 256; done
