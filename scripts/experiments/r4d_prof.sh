#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
export MIPIPE_GEMVS_S=${S:-16} MIPIPE_GEMVS_MINWG=${W:-256}
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/r4d_prof -o run -- python3 bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 10 --warmup 2 > $O/r4d_prof.log 2>&1 || { tail -5 $O/r4d_prof.log; exit 1; }
echo done
