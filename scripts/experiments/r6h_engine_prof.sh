#!/bin/bash
# in-engine kernel times of gemm3 vs gemm2 (70B mb256); HIP failover/elastic tests; 8B single-stream profile
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for v in 3 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r6h_prof_v$v -o run -- python bench.py --steps 10 --warmup 2 \
    --no-secondary --set prefill_gemm_v=$v > $O/r6h_bench_v$v.log 2>&1 || { tail -5 $O/r6h_bench_v$v.log; exit 1; }
  echo "v$v $(grep -o '"value": [0-9.]*' $O/r6h_bench_v$v.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r6h_prof8b -o run -- python bench.py --model llama3-8b --ftype Q4_K_M \
  --mb-size 1 --steps 20 --warmup 3 --no-secondary > $O/r6h_bench8b_mb1.log 2>&1 || { tail -5 $O/r6h_bench8b_mb1.log; exit 1; }
echo "8b mb1 $(grep -o '"value": [0-9.]*' $O/r6h_bench8b_mb1.log)"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_failover_gpu.py > $O/r6h_failover.log 2>&1 || { tail -40 $O/r6h_failover.log; exit 1; }
grep -E "passed|failed" $O/r6h_failover.log | tail -3
