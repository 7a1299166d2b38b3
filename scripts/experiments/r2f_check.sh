set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemv_fused_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2f_tests.log 2>&1 || { tail -40 gpurun_out/r2f_tests.log; exit 1; }
tail -2 gpurun_out/r2f_tests.log
timeout -k 10 150 python tools/gemv_bench.py --shapes 8b.qkv,8b.o,8b.gateup,8b.down,70b.gateup,70b.down --types Q4_K,Q6_K --M 1 --splits 1,2,4,8 > gpurun_out/r2f_gemv_m1.log 2>&1 || exit 1
timeout -k 10 150 python tools/gemv_bench.py --shapes 70b.qkv,70b.o,70b.gateup,70b.down --types Q4_K --M 64 > gpurun_out/r2f_gemv_m64.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 50 > gpurun_out/r2f_bench8b.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 50 --set fused_norm=false > gpurun_out/r2f_bench8b_nofuse.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mb-size 1 --steps 20 > gpurun_out/r2f_bench70b_mb1.log 2>&1 || exit 1
timeout -k 10 200 python bench.py > gpurun_out/r2f_bench70b_mb64.log 2>&1 || exit 1
