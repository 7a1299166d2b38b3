set -o pipefail
mkdir -p gpurun_out
for ns in 4 8; do
  MIPIPE_GEMV3_NS=$ns timeout -k 10 150 python tools/gemv_bench.py --shapes 8b.gateup,8b.down,70b.gateup,70b.down,8b.qkv --types Q4_K --M 1 --splits 1,2,4,8 > gpurun_out/r2e_gemv_ns$ns.log 2>&1 || exit 1
done
