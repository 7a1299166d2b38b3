#!/bin/bash
# r12i: 96-row MoE expert tiles (GEMM4_MOE64=2) -- oracle tests, Mixtral mb256 A/B and kernel summary
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_moe_gemm_gpu.py \
  "tests/test_engine_gpu.py::test_moe_grouped_gemm_matches_slices_and_reference" > $O/r12i_tests.log 2>&1; rc=$?; tail -4 $O/r12i_tests.log; [ $rc -ne 0 ] && exit $rc
run() { local n=$1 e="$2"; shift 2; timeout -k 10 300 env $e python3 -u $R/bench.py --no-secondary "$@" > $O/r12i_$n.log 2>&1 || { tail -5 $O/r12i_$n.log; exit 1; }
  echo "== $n $(grep -o '"value": [0-9.]*' $O/r12i_$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r12i_$n.log)"; }
run mix_t128 "MIPIPE_GEMM4_MOE64=0" --model mixtral-8x7b --ftype Q4_K_M --mb-size 256
run mix_t96 "MIPIPE_GEMM4_MOE64=2" --model mixtral-8x7b --ftype Q4_K_M --mb-size 256
run mix_t128b "MIPIPE_GEMM4_MOE64=0" --model mixtral-8x7b --ftype Q4_K_M --mb-size 256
run mix_t96b "MIPIPE_GEMM4_MOE64=2" --model mixtral-8x7b --ftype Q4_K_M --mb-size 256
cd /tmp
export MIPIPE_GEMM4_MOE64=2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r12i_prof -- python3 $R/bench.py --steps 30 --warmup 3 --no-secondary --model mixtral-8x7b --ftype Q4_K_M --mb-size 256 > $O/r12i_prof.log 2>&1 || { tail -3 $O/r12i_prof.log; exit 1; }
python3 $R/tools/prof_summary.py $O/r12i_prof > $O/r12i_prof_mixtral_t96.txt; rm -rf $O/r12i_prof; sed -n '/last 5 decode/,/dispatch order/p' $O/r12i_prof_mixtral_t96.txt | head -12
