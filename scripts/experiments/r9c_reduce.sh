#!/bin/bash
# r9c: split-K partial reductions (RMSNorm-fused and standalone) issue every split's loads before the
# first add: tests, then engine A/B against the previous build (lib/libmipipe_old.so) + kernel trace
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 600 python -u -m pytest -q --timeout 250 --timeout-method thread -m gpu -p no:cacheprovider"
$T tests/test_deterministic_gpu.py tests/test_gemm2_gpu.py tests/test_kernels_gpu.py > $O/r9c_t.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" $O/r9c_t.log | tail -4; [ $rc -ne 0 ] && exit $rc
$T tests/test_engine_gpu.py -k "70b or wide or split" > $O/r9c_t2.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" $O/r9c_t2.log | tail -4; [ $rc -ne 0 ] && exit $rc
BB="timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-secondary"
for rep in 1 2; do for lib in new old; do
  if [ $lib = old ]; then export MIPIPE_LIB=libmipipe_old.so; else unset MIPIPE_LIB; fi
  $BB > $O/r9c_70_$lib.log 2>&1 || { tail -3 $O/r9c_70_$lib.log; exit 1; }
  echo "rep $rep $lib: 70b mb256 $(grep -o '"value": [0-9.]*' $O/r9c_70_$lib.log)"
done; done
unset MIPIPE_LIB
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r9c_p -- python3 $R/bench.py --steps 10 --warmup 2 --no-secondary > $O/r9c_p.log 2>&1 || exit 1
python3 $R/tools/prof_summary.py $O/r9c_p > $O/r9c_p.txt; rm -rf $O/r9c_p; sed -n '/last 5 decode/,/dispatch order/p' $O/r9c_p.txt | head -8
