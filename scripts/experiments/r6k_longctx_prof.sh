#!/bin/bash
# 70B mb256 at 2K context: kernel profile (summary made on the box; the db exceeds the copy-back cap); bf16 8B after the staging change
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for kv in f16 fp8; do
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r6k_prof_$kv -o run -- python bench.py --steps 6 --warmup 1 --no-secondary \
  --prompt-len 2040 --mb-size 256 --set kv_dtype=$kv > $O/r6k_bench_$kv.log 2>&1 || { tail -5 $O/r6k_bench_$kv.log; exit 1; }
python tools/prof_db_summary.py $O/r6k_prof_$kv 3 > $O/r6k_prof_$kv.txt; rm -rf $O/r6k_prof_$kv
head -8 $O/r6k_prof_$kv.txt
done
for mb in 1 64; do
  timeout -k 10 300 python bench.py --model llama3-8b --ftype BF16 --mb-size $mb --steps 20 --warmup 3 --no-secondary \
    > $O/r6k_bf16_mb$mb.log 2>&1 || { tail -5 $O/r6k_bf16_mb$mb.log; exit 1; }
  echo "bf16 mb$mb $(grep -o '"value": [0-9.]*' $O/r6k_bf16_mb$mb.log)"
done
