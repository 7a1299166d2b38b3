#!/bin/bash
# int8_gemm with the RMSNorm emitting the int8 rows: tests, bench A/B, then a gemm3<P_I8> tile sweep
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gemm_i8_gpu.py tests/test_engine_gpu.py -q -x -s -k "i8 or int8 or 70b_width or wide" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_i8.log 2>&1; rc=$?
grep -E "int8_gemm NMSE|passed|failed" $O/t_i8.log | tail -4
[ $rc -ne 0 ] && exit $rc
for i8 in false true false true; do
  timeout -k 10 300 python bench.py --steps 15 --warmup 3 --no-secondary --set int8_gemm=$i8 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "int8_gemm=$i8 $(grep -o '"value": [0-9.]*' $O/b.log)"
done
bash scripts/experiments/r7m_i8_tiles.sh
