#!/bin/bash
# int8_gemm engine mode (K15): int8 kernel tests + the 70B-width oracle test, then bench A/B (exact f16 vs int8)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gemm_i8_gpu.py tests/test_engine_gpu.py -q -x -s -k "i8 or int8" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_i8.log 2>&1; rc=$?
grep -E "NMSE|passed|failed" $O/t_i8.log | tail -12
[ $rc -ne 0 ] && exit $rc
for args in "" "--model llama3-8b --ftype Q4_K_M" "--mb-size 512"; do
  for i8 in false true; do
    timeout -k 10 300 python bench.py --steps 15 --warmup 3 --no-secondary $args --set int8_gemm=$i8 > $O/b.log 2>&1 \
      || { tail -5 $O/b.log; exit 1; }
    echo "[$args] int8_gemm=$i8 $(grep -o '"value": [0-9.]*' $O/b.log) $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  done
done
