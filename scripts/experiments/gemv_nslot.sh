#!/bin/bash
# per-type NSLOT (Q6_K/Q8_0 3, F16 2): kernel tests + microbench + 8B/70B benches
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/nslot; mkdir -p $O; cd $R
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -p no:cacheprovider > $O/kt.log 2>&1; rc=$?; tail -1 $O/kt.log
grep -E "^FAILED" $O/kt.log | head -5
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/gemv_bench.py --types Q6_K,Q8_0,F16 --M 1,16 --tpw 1 --target 4096 --shapes 70b.qkv,70b.o,70b.gateup,70b.down,70b.head > $O/mb.log 2>&1 || { tail -3 $O/mb.log; exit 1; }
grep shape $O/mb.log | sed -E 's/.*"shape": "([^"]+)", "type": "([^"]+)".*"M": ([0-9]+).*"us": ([0-9.]+), "GBps": ([0-9.]+).*/\1 \2 M\3 \4us \5GB\/s/'
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/b16.log 2>&1 || { tail -5 $O/b16.log; exit 1; }
grep '"value"' $O/b16.log | cut -c1-110
timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --steps 30 --warmup 3 --mb-size 1 > $O/b8.log 2>&1 || { tail -5 $O/b8.log; exit 1; }
grep '"value"' $O/b8.log | cut -c1-110
timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --steps 30 --warmup 3 > $O/b8_16.log 2>&1 || { tail -5 $O/b8_16.log; exit 1; }
grep '"value"' $O/b8_16.log | cut -c1-110
