#!/bin/bash
# r8a: gemm4 (32x32x16) first light: oracle tests, micro-bench vs gemm2 / gemm3 at M=256, engine A/B;
# wave-level decode attention tests + A/B; grouped MoE GEMM
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider"
[ -n "$WITH_G4" ] && { $T tests/test_gemm4_gpu.py > $O/r8a_t4.log 2>&1 || { tail -3 $O/r8a_t4.log; exit 1; }; }
$T tests/test_attn_wave_gpu.py > $O/r8a_ta.log 2>&1; rc=$?; tail -3 $O/r8a_ta.log; [ $rc -ne 0 ] && exit $rc
$T tests/test_engine_gpu.py -k "moe_grouped or inprocess or single_copy or 70b_width" > $O/r8a_te.log 2>&1; rc=$?; tail -3 $O/r8a_te.log; [ $rc -ne 0 ] && exit $rc
B="timeout -k 10 200 python -u tools/gemv_bench.py --M 256 --iters 20"
S=70b.qkv,70b.o,70b.gateup,70b.down,8b.gateup,8b.down
{ $B --gemm 2 --shapes $S && $B --gemm 2 --sk --shapes 70b.qkv,70b.o,70b.down,8b.down && \
  $B --gemm 3 --shapes $S && $B --gemm 4 --shapes $S && $B --gemm 4 --sk --shapes 70b.qkv,70b.o,70b.down,8b.down && \
  $B --gemm 4 --g3 "128,0,0" --shapes $S && $B --gemm 4 --shapes 70b.head --types Q6_K && $B --gemm 2 --shapes 70b.head --types Q6_K; } > $O/r8a_mb.log 2>&1 || { tail -5 $O/r8a_mb.log; exit 1; }
cut -c1-150 $O/r8a_mb.log
BB="timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-secondary"
$BB > $O/r8a_b2.log 2>&1 || { tail -5 $O/r8a_b2.log; exit 1; }
$BB --set prefill_gemm_v=4 > $O/r8a_b4.log 2>&1 || { tail -5 $O/r8a_b4.log; exit 1; }
MIPIPE_ATTN_WAVE=0 $BB --set prefill_gemm_v=4 > $O/r8a_b4nw.log 2>&1 || { tail -5 $O/r8a_b4nw.log; exit 1; }
$BB --model mixtral-8x7b --ftype Q4_K_M > $O/r8a_bmx.log 2>&1 || { tail -5 $O/r8a_bmx.log; exit 1; }
$BB --model mixtral-8x7b --ftype Q4_K_M --set moe_gemm=false > $O/r8a_bmx0.log 2>&1 || { tail -5 $O/r8a_bmx0.log; exit 1; }
grep -H -o '"value": [0-9.]*' $O/r8a_b*.log
