#!/bin/bash
# decode attention at 2K contexts: variant / split knobs (70B mb64 and mb256)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
run() {  # name, env..., then bench args
  local name=$1; shift
  timeout -k 10 400 env "$@" python bench.py --steps 6 --warmup 1 --no-secondary --prompt-len 2040 $BARGS > $O/r6l_$name.log 2>&1 \
    || { tail -5 $O/r6l_$name.log; exit 1; }
  echo "$name $(grep -o '"value": [0-9.]*' $O/r6l_$name.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r6l_$name.log)"
}
BARGS="--mb-size 64"
run mb64_default MIPIPE_X=0
run mb64_np MIPIPE_ATTN_PF_MAXWG=0
run mb64_wg2048 MIPIPE_ATTN_WG_TARGET=2048
run mb64_wg4096_np MIPIPE_ATTN_WG_TARGET=4096 MIPIPE_ATTN_PF_MAXWG=0
BARGS="--mb-size 256"
run mb256_np MIPIPE_ATTN_PF_MAXWG=0
run mb256_wg8192_np MIPIPE_ATTN_WG_TARGET=8192 MIPIPE_ATTN_PF_MAXWG=0
