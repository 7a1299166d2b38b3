#!/bin/bash
# r12b: (1) gemvs loads reordered (prologue inputs ahead of the weight ring), attn_o with separate DMA
# waves; (2) gemm4 8 / 7 waves x 64 columns on 128-row tiles (GEMM4_TW4 4 / 5 / 6) -- oracle tests,
# 8B mb1 kernel profile, 70B mb256 A/B
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemvs_gpu.py tests/test_gemm4_gpu.py \
  "tests/test_engine_gpu.py::test_engine_matches_reference" "tests/test_engine_gpu.py::test_fused_attention_o_matches_two_kernels" \
  "tests/test_engine_gpu.py::test_qkv_append_epilogue_matches_attention_append" "tests/test_engine_gpu.py::test_70b_width_mb256_matches_reference" \
  > $O/r12b_tests.log 2>&1; rc=$?; tail -4 $O/r12b_tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp
prof() { local n=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r12b_$n -- python3 $R/bench.py --steps 30 --warmup 3 --no-secondary "$@" > $O/r12b_$n.log 2>&1 || { tail -3 $O/r12b_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r12b_$n > $O/r12b_prof_$n.txt; rm -rf $O/r12b_$n; echo "== $n $(grep -o '"value": [0-9.]*' $O/r12b_$n.log)"; sed -n '/last 5 decode/,/dispatch order/p' $O/r12b_prof_$n.txt | head -12; }
prof 8b_mb1 --model llama3-8b --ftype Q4_K_M --mb-size 1
run() { local n=$1; shift; timeout -k 10 300 env "$@" python3 -u $R/bench.py --no-secondary > $O/r12b_$n.log 2>&1 || { tail -5 $O/r12b_$n.log; exit 1; }
  echo "== $n $(grep -o '"value": [0-9.]*' $O/r12b_$n.log)"; }
run 70b_tw1 MIPIPE_GEMM4_TW4=1
run 70b_tw4 MIPIPE_GEMM4_TW4=4
run 70b_tw5 MIPIPE_GEMM4_TW4=5
run 70b_tw6 MIPIPE_GEMM4_TW4=6
run 70b_tw1b MIPIPE_GEMM4_TW4=1
export MIPIPE_GEMM4_TW4=5; prof 70b_tw5 --model llama3-70b --ftype Q4_K --mb-size 256
unset MIPIPE_GEMM4_TW4
# pipeline rehearsal with LocalLink sends recorded on the compute stream (one hop fewer per item)
pp() { local n=$1; shift; timeout -k 10 300 python3 -u $R/bench.py --no-secondary "$@" > $O/r12b_$n.log 2>&1 || { tail -5 $O/r12b_$n.log; exit 1; }
  echo "== $n $(grep -o '"value": [0-9.]*' $O/r12b_$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r12b_$n.log)"; }
pp 8b_pp1 --model llama3-8b --ftype BF16 --mb-size 64
pp 8b_pp4 --model llama3-8b --ftype BF16 --mb-size 64 --gpus 4 --same-device --trace $O/r12b_8b_pp4.trace.json
