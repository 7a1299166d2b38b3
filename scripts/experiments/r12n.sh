#!/bin/bash
# r12n: MoE down split 4 over K on the 96-row tiles as the default (GEMM4_MOE64 2) vs unsplit (3)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_moe_gemm_gpu.py \
  "tests/test_engine_gpu.py::test_moe_grouped_gemm_matches_slices_and_reference" "tests/test_engine_gpu.py::test_moe_batched_matches_single" \
  tests/test_deterministic_gpu.py > $O/r12n_tests.log 2>&1; rc=$?; tail -3 $O/r12n_tests.log; [ $rc -ne 0 ] && exit $rc
run() { local n=$1 e="$2"; shift 2; timeout -k 10 300 env $e python3 -u $R/bench.py --no-secondary "$@" > $O/r12n_$n.log 2>&1 || { tail -5 $O/r12n_$n.log; exit 1; }
  echo "== $n $(grep -o '"value": [0-9.]*' $O/r12n_$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r12n_$n.log)"; }
for m in 2 3 2 3; do run mix_moe$m "MIPIPE_GEMM4_MOE64=$m" --model mixtral-8x7b --ftype Q4_K_M --mb-size 256; done
run mix64_moe2 "MIPIPE_GEMM4_MOE64=2" --model mixtral-8x7b --ftype Q4_K_M --mb-size 64
run mix64_moe3 "MIPIPE_GEMM4_MOE64=3" --model mixtral-8x7b --ftype Q4_K_M --mb-size 64
