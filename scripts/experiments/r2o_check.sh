#!/bin/bash
# prefill attention VALU trims + GGUF load at scale
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_attn_prefill_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r2o_tests.log 2>&1 || { tail -40 $O/r2o_tests.log; exit 1; }
tail -1 $O/r2o_tests.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pf_o -o run --output-format csv -- python3 $R/bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --prompt-len 32000 --steps 5 --warmup 1 > $O/pf_o.log 2>&1 || { tail -5 $O/pf_o.log; exit 1; }
python3 $R/tools/prof_summary.py $O/pf_o > $O/r2o_prof_8b_32k.txt || exit 1
head -6 $O/r2o_prof_8b_32k.txt
cd $R
timeout -k 10 600 python tools/load_bench.py --model llama3-8b --ftype Q4_K_M --out /tmp/mipipe_8b.gguf > $O/r2o_load_bench.log 2>&1 || { tail -20 $O/r2o_load_bench.log; exit 1; }
tail -1 $O/r2o_load_bench.log
