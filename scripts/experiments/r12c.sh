#!/bin/bash
# r12c: gemvs early loads with 2 slots (register budget restored), 8B mb1 profile; PP=8 70B rehearsal
# with compute-stream LocalLink sends
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemvs_gpu.py \
  "tests/test_engine_gpu.py::test_engine_matches_reference" "tests/test_engine_gpu.py::test_fused_attention_o_matches_two_kernels" \
  "tests/test_engine_gpu.py::test_qkv_append_epilogue_matches_attention_append" "tests/test_engine_gpu.py::test_local_link_posted_queue_delayed_receiver" \
  "tests/test_engine_gpu.py::test_pipeline_emulation_matches_pp1" "tests/test_engine_gpu.py::test_bench_inprocess_same_device" \
  > $O/r12c_tests.log 2>&1; rc=$?; tail -4 $O/r12c_tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp
prof() { local n=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r12c_$n -- python3 $R/bench.py --steps 30 --warmup 3 --no-secondary "$@" > $O/r12c_$n.log 2>&1 || { tail -3 $O/r12c_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r12c_$n > $O/r12c_prof_$n.txt; rm -rf $O/r12c_$n; echo "== $n $(grep -o '"value": [0-9.]*' $O/r12c_$n.log)"; sed -n '/last 5 decode/,/dispatch order/p' $O/r12c_prof_$n.txt | head -12; }
prof 8b_mb1 --model llama3-8b --ftype Q4_K_M --mb-size 1
pp() { local n=$1; shift; timeout -k 10 300 python3 -u $R/bench.py --no-secondary "$@" > $O/r12c_$n.log 2>&1 || { tail -5 $O/r12c_$n.log; exit 1; }
  echo "== $n $(grep -o '"value": [0-9.]*' $O/r12c_$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r12c_$n.log)"; }
pp 70b_pp1 --model llama3-70b --ftype Q4_K --mb-size 256
pp 70b_pp8 --model llama3-70b --ftype Q4_K --mb-size 256 --gpus 8 --same-device
pp 8b_pp1 --model llama3-8b --ftype BF16 --mb-size 64
pp 8b_pp4 --model llama3-8b --ftype BF16 --mb-size 64 --gpus 4 --same-device
pp 8b_q4_pp1 --model llama3-8b --ftype Q4_K_M --mb-size 1
