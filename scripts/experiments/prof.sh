#!/bin/bash
# rocprofv3 kernel trace + stats for the 1-GPU bench at mb_size 16 and 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof16 $R/gpurun_out/prof1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof16 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --mb-size 16 > $R/gpurun_out/prof16.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --mb-size 1 > $R/gpurun_out/prof1.log 2>&1 || exit $?
tail -2 $R/gpurun_out/prof16.log $R/gpurun_out/prof1.log
find $R/gpurun_out/prof16 -name "*stats*"
