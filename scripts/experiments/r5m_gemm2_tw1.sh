#!/bin/bash
# gemm2: one tile per wave when a non-split grid has fewer two-tile workgroups than CUs
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_kernels_gpu.py tests/test_prefill.py tests/test_engine_gpu.py > $O/r5m_tests.log 2>&1 || { tail -30 $O/r5m_tests.log; exit 1; }
tail -1 $O/r5m_tests.log
for cfg in "llama3-8b Q4_K_M 256" "llama3-8b Q4_K_M 128" "llama3-70b Q4_K 128"; do
  set -- $cfg
  for t in 0 256; do
    MIPIPE_GEMM2_TW1_BELOW=$t timeout -k 10 300 python bench.py --model $1 --ftype $2 --mb-size $3 --steps 10 --warmup 2 > $O/r5m.log 2>&1 || { tail -5 $O/r5m.log; exit 1; }
    echo "tw1_below=$t $1 mb$3 $(grep -o '"value": [0-9.]*' $O/r5m.log)"
  done
done
