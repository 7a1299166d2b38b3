set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemv3_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2d_tests.log 2>&1 || { tail -30 gpurun_out/r2d_tests.log; exit 1; }
tail -2 gpurun_out/r2d_tests.log
for cfg in "v3nw4:MIPIPE_GEMV3_NW=4" "v3nw8:MIPIPE_GEMV3_NW=8" "v2:MIPIPE_GEMV_V3=0"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 150 python tools/gemv_bench.py --shapes 8b.qkv,8b.o,8b.gateup,8b.down,70b.gateup,70b.down --types Q4_K,Q6_K --M 1 --splits 1,2,4,8 > gpurun_out/r2d_gemv_$name.log 2>&1 || exit 1
done
for cfg in "v3:MIPIPE_GEMV3_NW=4" "v3nw8:MIPIPE_GEMV3_NW=8" "v2:MIPIPE_GEMV_V3=0"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 200 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 50 > gpurun_out/r2d_bench8b_$name.log 2>&1 || exit 1
done
