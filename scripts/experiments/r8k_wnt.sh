#!/bin/bash
# r8k: non-temporal weight LDS-DMA in gemm4 (knob GEMM4_WNT), one-row router workgroups; engine kernel traces
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 400 python -u -m pytest -q -x --timeout 250 --timeout-method thread -m gpu -p no:cacheprovider"
MIPIPE_GEMM4_WNT=1 $T tests/test_gemm4_gpu.py tests/test_moe_gemm_gpu.py -k "tiles or headline or mixtral or router" > $O/r8k_t.log 2>&1; rc=$?; tail -2 $O/r8k_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/gemv_bench.py --M 256 --iters 20 --gemm 4 --shapes 70b.gateup,8b.gateup,70b.head --knob GEMM4_WNT=0,1 > $O/r8k_mb.log 2>&1 || { tail -5 $O/r8k_mb.log; exit 1; }
grep shape $O/r8k_mb.log | cut -c1-110
cd /tmp
P="timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -o run"
pr() { local n=$1; shift; $P -d $O/r8k_$n -- python3 $R/bench.py --steps 6 --warmup 2 --no-secondary "$@" > $O/r8k_$n.log 2>&1 || { tail -3 $O/r8k_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r8k_$n > $O/r8k_$n.txt; echo "== $n $(grep -o '"value": [0-9.]*' $O/r8k_$n.log)"; sed -n '/last 5 decode/,/dispatch order/p' $O/r8k_$n.txt | head -9 | cut -c1-120; }
export MIPIPE_GEMM4_WNT=1; pr 70nt; pr mxnt --model mixtral-8x7b --ftype Q4_K_M; unset MIPIPE_GEMM4_WNT
pr mx0 --model mixtral-8x7b --ftype Q4_K_M
MIPIPE_GEMM4_WNT=1 timeout -k 10 300 python3 $R/bench.py --steps 10 --warmup 3 --no-secondary > $O/r8k_b70nt.log 2>&1; timeout -k 10 300 python3 $R/bench.py --steps 10 --warmup 3 --no-secondary > $O/r8k_b70.log 2>&1; grep -H -o "\"value\": [0-9.]*" $O/r8k_b70*.log
