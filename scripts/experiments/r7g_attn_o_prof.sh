#!/bin/bash
# dispatch-order profile of the 8B mb1 round with the fused attention + o-projection kernel
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ao -o run --output-format csv -- \
  python3 $R/bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 30 --warmup 3 --no-secondary --set attn_o_max_ctx=4096 \
  > $O/prof_ao.log 2>&1 || { tail -5 $O/prof_ao.log; exit 1; }
PROF_SEQ=12 python3 $R/tools/prof_summary.py $O/prof_ao > $O/prof_8b_mb1_attn_o.txt && tail -24 $O/prof_8b_mb1_attn_o.txt
rm -rf $O/prof_ao
