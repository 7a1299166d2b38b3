#!/bin/bash
# r10ah: the new 4-wave oracle tests; the LM head with / without the 4-wave form; 8B single-stream gemvs G / split sweep
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gemm4_gpu.py -k four_wave > $O/r10ah_t.log 2>&1 || { tail -30 $O/r10ah_t.log; exit 1; }
tail -1 $O/r10ah_t.log
bash scripts/experiments/r10ag.sh
