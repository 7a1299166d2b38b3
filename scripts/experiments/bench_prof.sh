#!/bin/bash
# quick: GPU tests, bench (mb16, mb1), kernel-trace of a short bench (decode rounds summary)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -m pytest tests -q -m gpu -x -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 2>&1 | grep '"value"' | tee $O/bench16.json || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --mb-size 1 2>&1 | grep '"value"' | tee $O/bench1.json || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 8 --warmup 2 --prompt-len 16 > $O/prof.log 2>&1 || exit $?
python3 $R/tools/trace_summary.py $(ls $O/prof/*/run_kernel_trace.csv $O/prof/run_kernel_trace.csv 2>/dev/null | head -1) 5
