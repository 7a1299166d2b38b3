#!/bin/bash
# gemvs plan sweep on 70B single stream (the 8B sweep chose S=16, MINWG=256)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for cfg in "16 256" "8 256" "32 256" "16 512" "8 512"; do
  set -- $cfg
  MIPIPE_GEMVS_S=$1 MIPIPE_GEMVS_MINWG=$2 timeout -k 10 300 python bench.py --mb-size 1 --steps 20 --warmup 3 > $O/r5g_$1_$2.log 2>&1 || { tail -5 $O/r5g_$1_$2.log; exit 1; }
  echo "S=$1 MINWG=$2 70b mb1 $(grep -o '"value": [0-9.]*' $O/r5g_$1_$2.log)"
done
