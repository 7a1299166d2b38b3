#!/bin/bash
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/fast; mkdir -p $O; cd $R
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -p no:cacheprovider -k "gemv or gemm" > $O/kt.log 2>&1; rc=$?; tail -2 $O/kt.log
[ $rc -gt 1 ] && exit $rc
grep -E "FAILED|assert" $O/kt.log | head -8
for F in 0 1; do
  MIPIPE_GEMV_FAST=$F timeout -k 10 200 python tools/gemv_bench.py --types Q4_K --M 1,16 --tpw 1 --target 4096 > $O/f$F.log 2>&1 || { tail -3 $O/f$F.log; exit 1; }
done
paste <(grep shape $O/f0.log | sed -E 's/.*"shape": "([^"]+)".*"M": ([0-9]+).*"us": ([0-9.]+).*/\1 M\2 \3/') <(grep shape $O/f1.log | sed -E 's/.*"us": ([0-9.]+), "GBps": ([0-9.]+).*/fast \1 \2GB\/s/')
for F in 0 1; do MIPIPE_GEMV_FAST=$F timeout -k 10 300 python bench.py --steps 20 --warmup 3 2>&1 | grep '"value"' | cut -c1-110; done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --mb-size 1 2>&1 | grep '"value"' | cut -c1-110
timeout -k 10 400 python -m pytest tests/test_engine_gpu.py -q -m gpu -p no:cacheprovider -x > $O/et.log 2>&1; tail -2 $O/et.log
