#!/bin/bash
# r8j: gemm4 with 3-5 stage buffers (128-row tiles: 4-5), second attention chunk preloaded; tests,
# engine A/B (MoE row tile), kernel traces, attention stamps, the driver's default bench line
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 500 python -u -m pytest -q -x --timeout 250 --timeout-method thread -m gpu -p no:cacheprovider"
$T tests/test_gemm4_gpu.py tests/test_moe_gemm_gpu.py tests/test_attn_wave_gpu.py > $O/r8j_t.log 2>&1; rc=$?; tail -2 $O/r8j_t.log; grep MISMATCH $O/r8j_t.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
$T tests/test_engine_gpu.py -k "moe or 70b_width or decode or reference" > $O/r8j_te.log 2>&1; rc=$?; tail -2 $O/r8j_te.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/gemv_bench.py --M 256 --iters 20 --gemm 4 --shapes 8b.gateup,70b.gateup --g3 "128,0,0" > $O/r8j_mb.log 2>&1 || { tail -5 $O/r8j_mb.log; exit 1; }
grep shape $O/r8j_mb.log | cut -c1-120
cd /tmp
P="timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -o run"
pr() { local n=$1; shift; $P -d $O/r8j_$n -- python3 $R/bench.py --steps 6 --warmup 2 --no-secondary "$@" > $O/r8j_$n.log 2>&1 || { tail -3 $O/r8j_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r8j_$n > $O/r8j_$n.txt; echo "== $n $(grep -o '"value": [0-9.]*' $O/r8j_$n.log)"; sed -n '/last 5 decode/,/dispatch order/p' $O/r8j_$n.txt | head -7 | cut -c1-120; }
pr mx64 --model mixtral-8x7b --ftype Q4_K_M
export MIPIPE_GEMM3_BM=128; pr mx128 --model mixtral-8x7b --ftype Q4_K_M; unset MIPIPE_GEMM3_BM
pr 8b1 --model llama3-8b --ftype Q4_K_M --mb-size 1
cd $R
MIPIPE_LIB=../lib_probes/libmipipe.so MIPIPE_ATTN_PROBE=4 timeout -k 10 200 python3 bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --no-secondary --steps 3 --warmup 1 --no-graphs > $O/r8j_stamps.log 2>&1 || { tail -3 $O/r8j_stamps.log; exit 1; }
grep "attn stamps" $O/r8j_stamps.log | head -4
t0=$(date +%s); timeout -k 10 600 python3 bench.py > $O/r8j_bench.log 2>&1 || { tail -3 $O/r8j_bench.log; exit 1; }; echo "bench wall $(( $(date +%s) - t0 )) s"
tail -1 $O/r8j_bench.log | cut -c1-3000
