#!/bin/bash
# 70B Q4_K at 2048-token contexts (the reference's -c 2048): mb64 / mb256, f16 and fp8 KV; kernel profile of mb256 f16
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for mb in 64 256; do for kv in f16 fp8; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-secondary --prompt-len 2040 --mb-size $mb \
    --set kv_dtype=$kv > $O/r6g_ctx2k_mb${mb}_$kv.log 2>&1 || { tail -5 $O/r6g_ctx2k_mb${mb}_$kv.log; exit 1; }
  echo "mb$mb $kv $(grep -o '"value": [0-9.]*' $O/r6g_ctx2k_mb${mb}_$kv.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r6g_ctx2k_mb${mb}_$kv.log)"
done; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r6g_prof -o run -- python bench.py --steps 10 --warmup 2 --no-secondary \
  --prompt-len 2040 --mb-size 256 > $O/r6g_prof_bench.log 2>&1 || { tail -5 $O/r6g_prof_bench.log; exit 1; }
python tools/prof_db_summary.py $O/r6g_prof 3 > $O/r6g_prof_summary.txt && rm -rf $O/r6g_prof   # the db exceeds the copy-back cap
head -12 $O/r6g_prof_summary.txt
