#!/bin/bash
# r10m: gemm4 with the spread fragment schedule (Q4_K + Q6_K): oracle tests; then 64-row micro-batches
# on gemm4 (r10i) and the MoE weight-DMA A/B (r10f)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gemm4_gpu.py tests/test_moe_gemm_gpu.py > $O/r10m_t.log 2>&1 || { tail -30 $O/r10m_t.log; exit 1; }
tail -1 $O/r10m_t.log
bash scripts/experiments/r10i.sh && bash scripts/experiments/r10f.sh
