#!/bin/bash
# r12f: decode GEMV (M = 64) forms A/B: GEMV_NW (waves per workgroup) x GEMV2_TW (tiles per wave) on 70B Q4_K and 8B BF16 mb64
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
run() { local n=$1 e="$2"; shift 2; timeout -k 10 300 env $e python3 -u $R/bench.py --no-secondary --mb-size 64 "$@" > $O/r12f_$n.log 2>&1 || { tail -5 $O/r12f_$n.log; exit 1; }
  echo "== $n $(grep -o '"value": [0-9.]*' $O/r12f_$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r12f_$n.log)"; }
for cfg in 8:0 4:0 8:2 4:2 8:1; do
  nw=${cfg%:*}; tw=${cfg#*:}
  run 70b_nw${nw}_tw${tw} "MIPIPE_GEMV_NW=$nw MIPIPE_GEMV2_TW=$tw" --model llama3-70b --ftype Q4_K
done
for cfg in 8:0 4:0; do
  nw=${cfg%:*}; tw=${cfg#*:}
  run 8b_nw${nw}_tw${tw} "MIPIPE_GEMV_NW=$nw MIPIPE_GEMV2_TW=$tw" --model llama3-8b --ftype BF16
done
