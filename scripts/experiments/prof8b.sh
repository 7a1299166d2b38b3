#!/bin/bash
# rocprofv3 kernel stats of the 8B Q4_K_M mb1 bench + 70B PP=1 with 2 micro-batches in flight
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8 -o run --output-format csv -- python3 $R/bench.py --model llama3-8b --ftype Q4_K_M --steps 10 --warmup 2 --mb-size 1 > $O/prof8.log 2>&1 || { tail -5 $O/prof8.log; exit 1; }
python3 $R/tools/prof_summary.py $O/prof8 > $O/prof_8b_mb1.txt && cat $O/prof_8b_mb1.txt
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --n-mb 2 > $O/b70_nmb2.log 2>&1 || { tail -5 $O/b70_nmb2.log; exit 1; }
grep '"value"' $O/b70_nmb2.log
