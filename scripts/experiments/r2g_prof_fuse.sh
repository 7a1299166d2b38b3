#!/bin/bash
# rocprofv3 kernel stats of 8B Q4_K_M mb1: fused RMSNorm (default) vs unfused
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
for v in fuse nofuse; do
  extra=""; [ $v = nofuse ] && extra="--set fused_norm=false"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p8_$v -o run --output-format csv -- python3 $R/bench.py --model llama3-8b --ftype Q4_K_M --steps 10 --warmup 2 --mb-size 1 $extra > $O/p8_$v.log 2>&1 || { tail -5 $O/p8_$v.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/p8_$v > $O/r2g_prof_8b_mb1_$v.txt || exit 1
done
