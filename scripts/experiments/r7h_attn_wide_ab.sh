#!/bin/bash
# 70B mb256 decode attention variants at 128-153-token contexts: default (prefetch variant, one split),
# the 3-per-CU variant (MIPIPE_ATTN_PF_MAXWG=0), two KV splits (attn_split_len=128)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
run() {
  timeout -k 10 300 env "$@" python bench.py --steps 15 --warmup 3 --no-secondary > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
}
for i in 1 2; do
  run MIPIPE_X=0; echo "default $(grep -o '"value": [0-9.]*' $O/b.log)"
  run MIPIPE_ATTN_PF_MAXWG=0; echo "pf_off $(grep -o '"value": [0-9.]*' $O/b.log)"
  timeout -k 10 300 python bench.py --steps 15 --warmup 3 --no-secondary --set attn_split_len=128 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "split128 $(grep -o '"value": [0-9.]*' $O/b.log)"
done
