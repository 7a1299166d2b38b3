#!/bin/bash
# iteration check: GPU tests, GEMV A/B (MIPIPE_GEMV_XR = fast-dequant experiment), 70B bench
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/iter; mkdir -p $O; cd $R
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" $O/tests.log | tail -12
[ $rc -gt 1 ] && exit $rc
for XR in 0 1; do
  MIPIPE_GEMV_XR=$XR timeout -k 10 300 python tools/gemv_bench.py --types Q4_K --M 1,16 --tpw 1,2,4 > $O/time_xr$XR.log 2>&1 || { tail -3 $O/time_xr$XR.log; exit 1; }
done
paste <(grep shape $O/time_xr0.log | cut -c1-110) <(grep shape $O/time_xr1.log | sed -E 's/.*"us": ([0-9.]+).*/fast \1/')
timeout -k 10 300 python bench.py --steps 20 --warmup 3 2>&1 | grep '"value"' | cut -c1-200
MIPIPE_GEMV_XR=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 2>&1 | grep '"value"' | cut -c1-200
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --mb-size 1 2>&1 | grep '"value"' | cut -c1-200
