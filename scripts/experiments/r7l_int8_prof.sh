#!/bin/bash
# kernel profile of the 70B mb256 round in the int8_gemm mode
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_i8 -o run --output-format csv -- \
  python3 $R/bench.py --steps 8 --warmup 2 --no-secondary --set int8_gemm=true > $O/prof_i8.log 2>&1 || { tail -5 $O/prof_i8.log; exit 1; }
grep -o '"value": [0-9.]*' $O/prof_i8.log
PROF_SEQ=0 python3 $R/tools/prof_summary.py $O/prof_i8 > $O/prof_70b_mb256_int8.txt && tail -14 $O/prof_70b_mb256_int8.txt
rm -rf $O/prof_i8
