#!/bin/bash
# r12j: 96-row MoE tiles as the default (engine MoE tests, Mixtral secondary); dense 96-row tiles (GEMM3_BM=96) A/B
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_moe_gemm_gpu.py tests/test_gemm4_gpu.py \
  tests/test_engine_gpu.py tests/test_deterministic_gpu.py > $O/r12j_tests.log 2>&1; rc=$?; tail -4 $O/r12j_tests.log; [ $rc -ne 0 ] && exit $rc
run() { local n=$1 e="$2"; shift 2; timeout -k 10 300 env $e python3 -u $R/bench.py --no-secondary "$@" > $O/r12j_$n.log 2>&1 || { tail -5 $O/r12j_$n.log; exit 1; }
  echo "== $n $(grep -o '"value": [0-9.]*' $O/r12j_$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r12j_$n.log)"; }
run mix_default "MIPIPE_X=0" --model mixtral-8x7b --ftype Q4_K_M --mb-size 256
run 70b_bm0 "MIPIPE_GEMM3_BM=0"
run 70b_bm96 "MIPIPE_GEMM3_BM=96"
run 70b_bm0b "MIPIPE_GEMM3_BM=0"
run 70b_bm96b "MIPIPE_GEMM3_BM=96"
run 8b_bm0 "MIPIPE_GEMM3_BM=0" --model llama3-8b --ftype Q4_K_M --mb-size 256
run 8b_bm96 "MIPIPE_GEMM3_BM=96" --model llama3-8b --ftype Q4_K_M --mb-size 256
run mix64_default "MIPIPE_X=0" --model mixtral-8x7b --ftype Q4_K_M --mb-size 64
run mix64_t128 "MIPIPE_GEMM4_MOE64=0" --model mixtral-8x7b --ftype Q4_K_M --mb-size 64
