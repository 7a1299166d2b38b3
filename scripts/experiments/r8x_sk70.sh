#!/bin/bash
# r8x: gemm4 for the 70B decode split-K shapes (qkv / o / down, K and N >= 8192 at M <= 256;
# knob GEMM4_SK70=1 restores gemm2 there): the whole engine test file (the r8s failure came in-suite),
# then bench A/B; Mixtral with the 64-row MoE tile again now that gemm4's per-stage overhead is lower
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 700 python -u -m pytest -q --timeout 250 --timeout-method thread -m gpu -p no:cacheprovider"
$T tests/test_engine_gpu.py tests/test_gemm4_gpu.py > $O/r8x_t.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" $O/r8x_t.log | tail -4; [ $rc -ne 0 ] && exit $rc
BB="timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-secondary"
for rep in 1 2; do for sk in 0 1; do
  MIPIPE_GEMM4_SK70=$sk $BB > $O/r8x_70_$sk.log 2>&1 || { tail -3 $O/r8x_70_$sk.log; exit 1; }
  echo "rep $rep GEMM4_SK70=$sk: 70b mb256 $(grep -o '"value": [0-9.]*' $O/r8x_70_$sk.log)"
done; done
for m in 0 1; do
  MIPIPE_GEMM4_MOE64=$m $BB --model mixtral-8x7b --ftype Q4_K_M > $O/r8x_mx_$m.log 2>&1 || { tail -3 $O/r8x_mx_$m.log; exit 1; }
  echo "mixtral mb256 GEMM4_MOE64=$m $(grep -o '"value": [0-9.]*' $O/r8x_mx_$m.log)"
done
MIPIPE_GEMM4_MOE64=1 timeout -k 10 400 python -u -m pytest -q --timeout 250 --timeout-method thread -m gpu -p no:cacheprovider tests/test_moe_gemm_gpu.py > $O/r8x_t3.log 2>&1; grep -E "^FAILED|passed|failed" $O/r8x_t3.log | tail -3
