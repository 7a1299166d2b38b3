#!/bin/bash
# gemm3 split-shape tile rule A/B in the engine; 8B single-stream profile; HIP failover/elastic tests
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for v in 3 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-secondary --set prefill_gemm_v=$v > $O/r6f_bench_v$v.log 2>&1 \
    || { tail -5 $O/r6f_bench_v$v.log; exit 1; }
  echo "v$v $(grep -o '"value": [0-9.]*' $O/r6f_bench_v$v.log)"
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_failover_gpu.py > $O/r6f_failover.log 2>&1 || { tail -40 $O/r6f_failover.log; exit 1; }
grep -E "passed|failed" $O/r6f_failover.log | tail -3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r6f_prof8b -o run -- python bench.py --model llama3-8b --ftype Q4_K_M \
  --mb-size 1 --steps 20 --warmup 3 --no-secondary > $O/r6f_bench8b_mb1.log 2>&1 || { tail -5 $O/r6f_bench8b_mb1.log; exit 1; }
grep -o '"value": [0-9.]*' $O/r6f_bench8b_mb1.log
