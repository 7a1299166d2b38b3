#!/bin/bash
# tests (kernels+engine) -> bench (mb 16) -> rocprofv3 kernel stats of the bench
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 400 python -m pytest tests -q -m gpu -x -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 2>&1 | grep '"value"' | tee $O/bench16.json || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --mb-size 1 2>&1 | grep '"value"' | tee $O/bench1.json || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 > $O/prof.log 2>&1 || exit $?
python3 - <<PY
import csv,glob
f=glob.glob("$O/prof/**/run_kernel_stats.csv",recursive=True)[0]
rows=list(csv.DictReader(open(f)))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {100*float(r['TotalDurationNs'])/tot:5.1f}% calls={r['Calls']:>6} avg={float(r['AverageNs'])/1e3:8.1f}us  {r['Name'][:80]}")
PY
