#!/bin/bash
# rocprofv3 kernel stats of one bench config; usage: prof_mb.sh <tag> <bench args...>
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
T=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$T -o run --output-format csv -- python3 $R/bench.py "$@" > $O/prof_$T.log 2>&1 || { tail -5 $O/prof_$T.log; exit 1; }
python3 $R/tools/prof_summary.py $O/prof_$T > $O/prof_$T.txt && sed -n '/last 5 decode/,$p' $O/prof_$T.txt | head -12
grep -o '"value": [0-9.]*' $O/prof_$T.log
