#!/bin/bash
# prefill flash attention: oracle tests, engine tests, 8B 32K-prompt profile flash vs row-group kernel
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_attn_prefill_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r2m_tests.log 2>&1 || { tail -40 $O/r2m_tests.log; exit 1; }
tail -2 $O/r2m_tests.log
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_paged_kv.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r2m_tests2.log 2>&1 || { tail -40 $O/r2m_tests2.log; exit 1; }
tail -2 $O/r2m_tests2.log
cd /tmp
for v in true; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p32_$v -o run --output-format csv -- python3 $R/bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --prompt-len 32000 --steps 5 --warmup 1 --set prefill_flash=$v > $O/p32_$v.log 2>&1 || { tail -5 $O/p32_$v.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/p32_$v > $O/r2m_prof_8b_32k_flash_$v.txt || exit 1
done
