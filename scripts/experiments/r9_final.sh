#!/bin/bash
# r9: end-of-round check on the final tree: the whole GPU test suite, the driver's default bench line
# (all secondaries), smoke(), and a rocprofv3 kernel summary of the 70B headline
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/r9_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" $O/r9_tests.log | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r9_smoke.log 2>&1 || { tail -5 $O/r9_smoke.log; exit 1; }
tail -1 $O/r9_smoke.log
t0=$(date +%s); timeout -k 10 900 python3 bench.py > $O/r9_bench.log 2>&1 || { tail -5 $O/r9_bench.log; exit 1; }; echo "bench wall $(( $(date +%s) - t0 )) s"
tail -1 $O/r9_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step']); [print(k, v) for k,v in d.get('secondary',{}).items()]"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r9_p70 -- python3 $R/bench.py --steps 10 --warmup 2 --no-secondary > $O/r9_p70.log 2>&1 || exit 1
python3 $R/tools/prof_summary.py $O/r9_p70 > $O/r9_prof_70b_mb256.txt; rm -rf $O/r9_p70; sed -n '/last 5 decode/,/dispatch order/p' $O/r9_prof_70b_mb256.txt | head -12
