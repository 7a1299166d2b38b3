#!/bin/bash
# r10y: round-end bench -- the default bench line (with the secondaries), then a kernel summary of the headline config
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
timeout -k 10 500 python bench.py > $O/r10y_bench.log 2>&1 || { tail -5 $O/r10y_bench.log; exit 1; }
grep '"metric"' $O/r10y_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r10y_p -- python3 $R/bench.py --steps 10 --warmup 2 --no-secondary > $O/r10y_p.log 2>&1 || { tail -3 $O/r10y_p.log; exit 1; }
python3 $R/tools/prof_summary.py $O/r10y_p > $O/r10y_prof_70b_mb256.txt; rm -rf $O/r10y_p
echo "== prof $(grep -o '"value": [0-9.]*' $O/r10y_p.log)"; sed -n '/last 5 decode/,/dispatch order/p' $O/r10y_prof_70b_mb256.txt | head -12
