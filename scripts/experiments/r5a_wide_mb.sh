#!/bin/bash
# mb_size > 64 decode (gemm2 projections): GPU tests, then a 70B / 8B micro-batch sweep
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_deterministic_gpu.py tests/test_engine_gpu.py -k "deterministic or wide_microbatch" > $O/r5a_tests.log 2>&1 || { tail -30 $O/r5a_tests.log; exit 1; }
tail -3 $O/r5a_tests.log
for mb in 64 128 256 512; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --mb-size $mb > $O/r5a_70b_$mb.log 2>&1 || { tail -5 $O/r5a_70b_$mb.log; exit 1; }
  echo "70b mb$mb $(grep -o '"value": [0-9.]*, "unit"[^}]*"ms_per_step": [0-9.]*' $O/r5a_70b_$mb.log)"
done
for mb in 64 128 256 512; do
  timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --steps 10 --warmup 2 --mb-size $mb > $O/r5a_8b_$mb.log 2>&1 || { tail -5 $O/r5a_8b_$mb.log; exit 1; }
  echo "8b mb$mb $(grep -o '"value": [0-9.]*, "unit"[^}]*"ms_per_step": [0-9.]*' $O/r5a_8b_$mb.log)"
done
