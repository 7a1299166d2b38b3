#!/bin/bash
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/v2; mkdir -p $O; cd $R
for NW in 4 8; do
  MIPIPE_GEMV_NW=$NW timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -p no:cacheprovider -k "gemv" > $O/kt$NW.log 2>&1; rc=$?; tail -1 $O/kt$NW.log
  [ $rc -ne 0 ] && { grep -E "Error|assert" $O/kt$NW.log | head -5; exit $rc; }
done
MIPIPE_GEMV_V=1 timeout -k 10 200 python tools/gemv_bench.py --types Q4_K,Q6_K --M 1,16 --tpw 2,4 > $O/v1.log 2>&1 || { tail -3 $O/v1.log; exit 1; }
for NW in 4 8; do
  MIPIPE_GEMV_NW=$NW timeout -k 10 200 python tools/gemv_bench.py --types Q4_K,Q6_K --M 1,16 --tpw 1 --target 2048 > $O/v2_nw$NW.log 2>&1 || { tail -3 $O/v2_nw$NW.log; exit 1; }
  MIPIPE_GEMV_NW=$NW timeout -k 10 200 python tools/gemv_bench.py --types Q4_K --M 1,16 --tpw 1 --target 4096 > $O/v2_nw${NW}_t4k.log 2>&1 || { tail -3 $O/v2_nw${NW}_t4k.log; exit 1; }
done
cd $O; for f in v1.log v2_nw*.log; do echo "== $f"; grep shape $f | sed -E 's/.*"shape": "([^"]+)", "type": "([^"]+)".*"M": ([0-9]+), "tpw": ([0-9]), "nsplit": ([0-9]+), "us": ([0-9.]+), "GBps": ([0-9.]+).*/\1 \2 M\3 t\4 s\5 \6us \7/' | paste -sd'|' ; done
cd $R
for NW in 4 8; do MIPIPE_GEMV_NW=$NW timeout -k 10 300 python bench.py --steps 20 --warmup 3 2>&1 | grep '"value"' | cut -c1-120; done
MIPIPE_GEMV_NW=8 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --mb-size 1 2>&1 | grep '"value"' | cut -c1-120
MIPIPE_GEMV_NW=8 timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --steps 30 --warmup 3 --mb-size 1 2>&1 | grep '"value"' | cut -c1-120
