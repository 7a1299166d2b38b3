#!/bin/bash
# Fused RMSNorm validation: kernel + engine GPU tests, A/B bench (fused_norm on/off), mb1 bench.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/norm; mkdir -p $O; cd $R
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -m gpu -p no:cacheprovider -k "gemv or attention or rope or gemm" > $O/kt.log 2>&1; rc=$?; tail -2 $O/kt.log
grep -E "FAILED|Error" $O/kt.log | head -8
[ $rc -gt 1 ] && exit $rc
timeout -k 10 500 python -m pytest tests/test_engine_gpu.py -q -m gpu -p no:cacheprovider -x > $O/et.log 2>&1; rc=$?; tail -2 $O/et.log
grep -E "FAILED|Error" $O/et.log | head -8
[ $rc -gt 1 ] && exit $rc
for F in true false; do timeout -k 10 300 python bench.py --steps 20 --warmup 3 --set fused_norm=$F > $O/b_$F.log 2>&1 || { tail -5 $O/b_$F.log; exit 1; }; grep '"value"' $O/b_$F.log | cut -c1-120; done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --mb-size 1 > $O/b1.log 2>&1 || { tail -5 $O/b1.log; exit 1; }
grep '"value"' $O/b1.log | cut -c1-120
