#!/bin/bash
# r10af: decode GEMV split-K through partial stores + the next norm's reduction (GEMV_SKSTORE=1) vs float atomics (0):
# engine tests with the knob, then 70B mb64 / mb32 / mb16 and 8B mb64 A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
MIPIPE_GEMV_SKSTORE=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_engine_gpu.py > $O/r10af_t.log 2>&1 || { tail -30 $O/r10af_t.log; exit 1; }
tail -1 $O/r10af_t.log
for rep in 1 2; do
  for v in 0 1; do
    MIPIPE_GEMV_SKSTORE=$v timeout -k 10 200 python bench.py --mb-size 64 --steps 8 --warmup 2 --no-secondary > $O/r10af.log 2>&1 || { tail -3 $O/r10af.log; exit 1; }
    echo "rep $rep 70b mb64 GEMV_SKSTORE=$v $(grep -o '"value": [0-9.]*' $O/r10af.log)"
  done
done
for mb in 32 16; do
  for v in 0 1; do
    MIPIPE_GEMV_SKSTORE=$v timeout -k 10 200 python bench.py --mb-size $mb --steps 8 --warmup 2 --no-secondary > $O/r10af.log 2>&1 || { tail -3 $O/r10af.log; exit 1; }
    echo "70b mb$mb GEMV_SKSTORE=$v $(grep -o '"value": [0-9.]*' $O/r10af.log)"
  done
done
for v in 0 1; do
  MIPIPE_GEMV_SKSTORE=$v timeout -k 10 200 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 64 --steps 10 --warmup 2 --no-secondary > $O/r10af.log 2>&1 || { tail -3 $O/r10af.log; exit 1; }
  echo "8b mb64 GEMV_SKSTORE=$v $(grep -o '"value": [0-9.]*' $O/r10af.log)"
done
