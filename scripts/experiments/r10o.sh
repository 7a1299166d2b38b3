#!/bin/bash
# r10o: MALL prefetch side stream (knob PREFETCH) -- engine test, 8B / 70B single-stream A/B; then r10n
# (gemm4 4-stage ring at 128-row tiles, lib_b)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_prefetch_gpu.py > $O/r10o_t.log 2>&1 || { tail -30 $O/r10o_t.log; exit 1; }
tail -1 $O/r10o_t.log
for rep in 1 2; do
  for v in 0 128 256 512; do
    MIPIPE_PREFETCH=$v timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 32 --warmup 4 --no-secondary > $O/r10o_8b_$v.log 2>&1 || { tail -5 $O/r10o_8b_$v.log; exit 1; }
    echo "rep $rep 8b mb1 PREFETCH=$v $(grep -o '"value": [0-9.]*' $O/r10o_8b_$v.log)"
  done
done
for v in 0 256; do
  MIPIPE_PREFETCH=$v timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 4 --steps 32 --warmup 4 --no-secondary > $O/r10o_8b4_$v.log 2>&1 || exit 1
  echo "8b mb4 PREFETCH=$v $(grep -o '"value": [0-9.]*' $O/r10o_8b4_$v.log)"
done
bash scripts/experiments/r10n.sh
