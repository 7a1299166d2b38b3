#!/bin/bash
# prefill attention row groups per wave A/B (8B, 32K prompt), after the oracle tests
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_attn_prefill_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r2n_tests.log 2>&1 || { tail -40 $O/r2n_tests.log; exit 1; }
tail -1 $O/r2n_tests.log
cd /tmp
for rg in 1 2; do
  MIPIPE_PF_RG=$rg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pf_rg$rg -o run --output-format csv -- python3 $R/bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --prompt-len 32000 --steps 5 --warmup 1 > $O/pf_rg$rg.log 2>&1 || { tail -5 $O/pf_rg$rg.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/pf_rg$rg > $O/r2n_prof_8b_32k_rg$rg.txt || exit 1
  head -4 $O/r2n_prof_8b_32k_rg$rg.txt
done
