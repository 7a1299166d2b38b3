#!/bin/bash
# r12d: decode GEMV (M = 64) split-K target A/B: GEMV_SPLIT_WAVES x GEMV_SPLIT_MINSB on 8B BF16 and 70B Q4_K mb64
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
run() { local n=$1 e="$2"; shift 2; timeout -k 10 300 env $e python3 -u $R/bench.py --no-secondary --mb-size 64 "$@" > $O/r12d_$n.log 2>&1 || { tail -5 $O/r12d_$n.log; exit 1; }
  echo "== $n $(grep -o '"value": [0-9.]*' $O/r12d_$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r12d_$n.log)"; }
for cfg in 2048:4 1024:4 512:4 2048:8 256:4; do
  w=${cfg%:*}; s=${cfg#*:}
  run 8b_${w}_${s} "MIPIPE_GEMV_SPLIT_WAVES=$w MIPIPE_GEMV_SPLIT_MINSB=$s" --model llama3-8b --ftype BF16
done
for cfg in 2048:4 1024:4 512:4 2048:8; do
  w=${cfg%:*}; s=${cfg#*:}
  run 70b_${w}_${s} "MIPIPE_GEMV_SPLIT_WAVES=$w MIPIPE_GEMV_SPLIT_MINSB=$s" --model llama3-70b --ftype Q4_K
done
