#!/bin/bash
# r8s: gemm4 as the auto choice for every quantized wide GEMM: engine A/B against v2 (decode 70B /
# 8B mb256, Mixtral mb256; prompt processing 70B / 8B 64 x 512), gemm4 + engine tests
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 500 python -u -m pytest -q --timeout 250 --timeout-method thread -m gpu -p no:cacheprovider"
$T tests/test_engine_gpu.py tests/test_deterministic_gpu.py -k "70b_width or wide or moe or determin or prefill" > $O/r8s_t.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" $O/r8s_t.log | tail -4; [ $rc -gt 1 ] && exit $rc
BB="timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-secondary"
for v in 0 2; do
  $BB --set prefill_gemm_v=$v > $O/r8s_70_v$v.log 2>&1 || exit 1
  $BB --set prefill_gemm_v=$v --model llama3-8b --ftype Q4_K_M > $O/r8s_8_v$v.log 2>&1 || exit 1
  $BB --set prefill_gemm_v=$v --model mixtral-8x7b --ftype Q4_K_M > $O/r8s_mx_v$v.log 2>&1 || exit 1
  timeout -k 10 300 python3 tools/prefill_bench.py --set prefill_gemm_v=$v > $O/r8s_pf70_v$v.log 2>&1 || exit 1
  timeout -k 10 300 python3 tools/prefill_bench.py --model llama3-8b --ftype Q4_K_M --set prefill_gemm_v=$v > $O/r8s_pf8_v$v.log 2>&1 || exit 1
done
grep -H -o '"value": [0-9.]*' $O/r8s_*_v*.log
grep -H -o '"prompt_tok_s_wall": [0-9.]*' $O/r8s_pf*.log
