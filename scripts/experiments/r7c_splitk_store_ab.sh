#!/bin/bash
# A/B: M > 64 split-K GEMMs with float atomics (default) vs per-split partial stores + one reduction
# (gemm_splitk_store), 70B mb256 / mb512 and 8B mb256 decode, plus the all-rows oracle check
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 240 python -u scripts/diag_mb256.py /tmp/diag gemm_splitk_store=true > $O/diag_sk.log 2>&1 \
  || { tail -5 $O/diag_sk.log; exit 1; }
grep -E "run-to-run|failures" $O/diag_sk.log
for args in "" "--model llama3-8b --ftype Q4_K_M" "--mb-size 512"; do
  for sk in false true false true; do
    timeout -k 10 300 python bench.py --steps 15 --warmup 3 --no-secondary $args --set gemm_splitk_store=$sk > $O/b.log 2>&1 \
      || { tail -5 $O/b.log; exit 1; }
    echo "[$args] splitk_store=$sk $(grep -o '"value": [0-9.]*' $O/b.log) $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  done
done
