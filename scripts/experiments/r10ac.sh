#!/bin/bash
# r10ac: decode attention kernel choice at 64-row micro-batches: the wave kernel (one wave per (token, kv head)) from
# ATTN_WAVE_MIN (token, kv head) items down (default 1024 = mb128 at 8 kv heads) -- 70B Q4_K / 8B BF16 / 8B Q4_K_M at mb64, mb32
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
for rep in 1 2; do
  for v in 1024 128; do
    MIPIPE_ATTN_WAVE_MIN=$v timeout -k 10 300 python bench.py --mb-size 64 --steps 10 --warmup 3 --no-secondary > $O/r10ac_70b_$v.log 2>&1 || { tail -5 $O/r10ac_70b_$v.log; exit 1; }
    echo "rep $rep 70b mb64 ATTN_WAVE_MIN=$v $(grep -o '"value": [0-9.]*' $O/r10ac_70b_$v.log)"
  done
done
for v in 1024 128; do
  MIPIPE_ATTN_WAVE_MIN=$v timeout -k 10 300 python bench.py --model llama3-8b --ftype BF16 --mb-size 64 --steps 10 --warmup 3 --no-secondary > $O/r10ac_8bbf_$v.log 2>&1 || exit 1
  echo "8b bf16 mb64 ATTN_WAVE_MIN=$v $(grep -o '"value": [0-9.]*' $O/r10ac_8bbf_$v.log)"
  MIPIPE_ATTN_WAVE_MIN=$v timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 64 --steps 10 --warmup 3 --no-secondary > $O/r10ac_8b_$v.log 2>&1 || exit 1
  echo "8b q4km mb64 ATTN_WAVE_MIN=$v $(grep -o '"value": [0-9.]*' $O/r10ac_8b_$v.log)"
  MIPIPE_ATTN_WAVE_MIN=$v timeout -k 10 300 python bench.py --mb-size 32 --steps 10 --warmup 3 --no-secondary > $O/r10ac_70b32_$v.log 2>&1 || exit 1
  echo "70b mb32 ATTN_WAVE_MIN=$v $(grep -o '"value": [0-9.]*' $O/r10ac_70b32_$v.log)"
done
