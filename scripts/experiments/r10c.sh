#!/bin/bash
# r10c: TW=4 MoE tiles (oracle + Mixtral A/B), PP=8 same-device rehearsal (f32 / bf16 wire), RCCL
# CU-sharing proxy on the 70B GEMMs
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_moe_gemm_gpu.py tests/test_gemm4_gpu.py -k "mixtral or tail or qkv_width or tiles" > $O/r10c_t.log 2>&1 || { tail -20 $O/r10c_t.log; exit 1; }
tail -2 $O/r10c_t.log
for v in 0 2 0 2; do
  MIPIPE_GEMM4_MOE64=$v timeout -k 10 300 python bench.py --model mixtral-8x7b --ftype Q4_K_M --steps 10 --warmup 3 --no-secondary > $O/r10c_mx$v.log 2>&1 || { tail -5 $O/r10c_mx$v.log; exit 1; }
  echo "mixtral mb256 MOE64=$v $(grep -o '"value": [0-9.]*' $O/r10c_mx$v.log)"
done
MIPIPE_GEMM4_MOE64=2 timeout -k 10 300 python bench.py --model mixtral-8x7b --ftype Q4_K_M --mb-size 64 --steps 10 --warmup 3 --no-secondary > $O/r10c_mx64.log 2>&1 || exit 1
echo "mixtral mb64 MOE64=2 $(grep -o '"value": [0-9.]*' $O/r10c_mx64.log)"
bash scripts/experiments/r10b.sh || exit 1
timeout -k 10 300 python tools/gemv_bench.py --shapes 70b.gateup,70b.qkv,70b.down --M 256 --gemm 4 --sk --rccl-bytes 4194304 --iters 24 > $O/r10c_rccl.log 2>&1 || { tail -5 $O/r10c_rccl.log; exit 1; }
cat $O/r10c_rccl.log
