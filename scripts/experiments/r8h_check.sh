#!/bin/bash
# r8h: MoE oracle test x3 (intermittent down mismatch hunt), attention hoist check + 8B mb1 attention timing,
# gemm4 spread A/B, Mixtral mb256 / mb64 benches
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 300 python -u -m pytest -q -s --timeout 250 --timeout-method thread -m gpu -p no:cacheprovider"
for i in 1 2 3; do $T tests/test_moe_gemm_gpu.py > $O/r8h_tm$i.log 2>&1; echo "moe run $i rc=$? $(grep -E 'passed|failed' $O/r8h_tm$i.log | tail -1) $(grep MISMATCH $O/r8h_tm$i.log | cut -c1-300)"; done
$T tests/test_attn_wave_gpu.py tests/test_engine_gpu.py -x -k "attn or wave or decode or reference or fp8" > $O/r8h_ta.log 2>&1; rc=$?; tail -2 $O/r8h_ta.log; [ $rc -ne 0 ] && exit $rc
cd /tmp
P="timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -o run"
for c in 8 128; do
  $P -d $O/r8h_a$c -- python3 $R/bench.py --steps 20 --warmup 2 --no-secondary --model llama3-8b --ftype Q4_K_M --mb-size 1 --prompt-len $c > $O/r8h_a$c.log 2>&1 || exit 1
  python3 $R/tools/prof_summary.py $O/r8h_a$c > $O/r8h_a$c.txt; echo "ctx$c $(grep -o '"value": [0-9.]*' $O/r8h_a$c.log) $(grep -m3 attn_decode $O/r8h_a$c.txt | tail -1 | cut -c1-100)"
done
cd $R
timeout -k 10 200 python -u tools/gemv_bench.py --M 256 --iters 20 --gemm 4 --shapes 70b.gateup,8b.gateup,70b.head --knob GEMM4_SPREAD=0,1,2 > $O/r8h_spread.log 2>&1 || { tail -5 $O/r8h_spread.log; exit 1; }
grep shape $O/r8h_spread.log | cut -c1-160
BB="timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-secondary"
$BB --model mixtral-8x7b --ftype Q4_K_M > $O/r8h_bmx.log 2>&1 || { tail -5 $O/r8h_bmx.log; exit 1; }
$BB --model mixtral-8x7b --ftype Q4_K_M --mb-size 64 > $O/r8h_bmx64.log 2>&1 || { tail -5 $O/r8h_bmx64.log; exit 1; }
for sp in 0 1 2; do MIPIPE_GEMM4_SPREAD=$sp $BB > $O/r8h_b70_sp$sp.log 2>&1 || exit 1; done
grep -H -o '"value": [0-9.]*' $O/r8h_b*.log
