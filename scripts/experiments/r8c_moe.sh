#!/bin/bash
# r8c: 64-row MoE tile + dense router kernel: Mixtral-width oracle tests, engine MoE tests, Mixtral bench mb64 / mb256
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -p no:cacheprovider"
$T tests/test_moe_gemm_gpu.py > $O/r8c_tm.log 2>&1; rc=$?; tail -3 $O/r8c_tm.log; [ $rc -ne 0 ] && exit $rc
$T tests/test_engine_gpu.py -k "moe" tests/test_gemm4_gpu.py > $O/r8c_te.log 2>&1; rc=$?; tail -3 $O/r8c_te.log; [ $rc -ne 0 ] && exit $rc
BB="timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-secondary --model mixtral-8x7b --ftype Q4_K_M"
$BB > $O/r8c_bmx.log 2>&1 || { tail -5 $O/r8c_bmx.log; exit 1; }
$BB --mb-size 64 > $O/r8c_bmx64.log 2>&1 || { tail -5 $O/r8c_bmx64.log; exit 1; }
MIPIPE_GEMM3_BM=128 $BB > $O/r8c_bmx128.log 2>&1 || { tail -5 $O/r8c_bmx128.log; exit 1; }
grep -H -o '"value": [0-9.]*' $O/r8c_b*.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r8c_pmx -- python3 $R/bench.py --steps 6 --warmup 2 --no-secondary --model mixtral-8x7b --ftype Q4_K_M > $O/r8c_pmx.log 2>&1 || { tail -5 $O/r8c_pmx.log; exit 1; }
python3 $R/tools/prof_summary.py $O/r8c_pmx > $O/r8c_pmx.txt; sed -n 22,40p $O/r8c_pmx.txt
cd $R
timeout -k 10 200 python -u tools/gemv_bench.py --M 256 --iters 20 --gemm 4 --shapes 70b.gateup,8b.gateup,70b.head --knob GEMM4_SPREAD=0,1,2 > $O/r8c_spread.log 2>&1 || { tail -5 $O/r8c_spread.log; exit 1; }
grep shape $O/r8c_spread.log | cut -c1-200
for sp in 1 2; do MIPIPE_GEMM4_SPREAD=$sp timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-secondary > $O/r8c_b70_sp$sp.log 2>&1 || exit 1; done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-secondary > $O/r8c_b70_sp0.log 2>&1 || exit 1
grep -H -o '"value": [0-9.]*' $O/r8c_b70*.log
