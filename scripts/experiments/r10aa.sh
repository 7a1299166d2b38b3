#!/bin/bash
# r10aa: after the loop-exit drain fix -- gemm4 / MoE oracle tests (default: 4-wave gate/up tiles) and with the 4-wave
# form on every tile (GEMM4_TW4=2), then the 70B mb256 engine A/B of GEMM4_TW4 0 / 1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gemm4_gpu.py tests/test_moe_gemm_gpu.py > $O/r10aa_t.log 2>&1 || { tail -30 $O/r10aa_t.log; exit 1; }
tail -1 $O/r10aa_t.log
MIPIPE_GEMM4_TW4=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gemm4_gpu.py > $O/r10aa_t2.log 2>&1 || { tail -30 $O/r10aa_t2.log; exit 1; }
tail -1 $O/r10aa_t2.log
for rep in 1 2 3; do
  for v in 0 1; do
    MIPIPE_GEMM4_TW4=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-secondary > $O/r10aa_70b_$v.log 2>&1 || { tail -5 $O/r10aa_70b_$v.log; exit 1; }
    echo "rep $rep 70b mb256 GEMM4_TW4=$v $(grep -o '"value": [0-9.]*' $O/r10aa_70b_$v.log)"
  done
done
