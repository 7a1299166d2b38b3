#!/bin/bash
# r8b: auto GEMM choice per epilogue (v4 gate/up + head, v2 split-K) and the narrow-N gemm4 row tile;
# kernel traces of 70B mb256, Mixtral mb256, 8B mb1; PMC of the gemm4 gate/up at M = 256
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider"
$T tests/test_gemm4_gpu.py > $O/r8b_t4.log 2>&1 || { tail -5 $O/r8b_t4.log; exit 1; }
tail -1 $O/r8b_t4.log
timeout -k 10 200 python -u tools/gemv_bench.py --M 256 --iters 20 --gemm 4 --shapes 8b.gateup,70b.gateup > $O/r8b_mb.log 2>&1 || { tail -5 $O/r8b_mb.log; exit 1; }
cut -c1-120 $O/r8b_mb.log | grep shape
BB="timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-secondary"
$BB > $O/r8b_b70.log 2>&1 || { tail -5 $O/r8b_b70.log; exit 1; }
$BB --model mixtral-8x7b --ftype Q4_K_M --mb-size 64 > $O/r8b_bmx64.log 2>&1 || { tail -5 $O/r8b_bmx64.log; exit 1; }
grep -H -o '"value": [0-9.]*' $O/r8b_b*.log
P="timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run"
cd /tmp
$P -d $O/r8b_p70 -- python3 $R/bench.py --steps 6 --warmup 2 --no-secondary > $O/r8b_p70.log 2>&1 || { tail -5 $O/r8b_p70.log; exit 1; }
python3 $R/tools/prof_summary.py $O/r8b_p70 > $O/r8b_p70.txt
$P -d $O/r8b_pmx -- python3 $R/bench.py --steps 6 --warmup 2 --no-secondary --model mixtral-8x7b --ftype Q4_K_M > $O/r8b_pmx.log 2>&1 || { tail -5 $O/r8b_pmx.log; exit 1; }
python3 $R/tools/prof_summary.py $O/r8b_pmx > $O/r8b_pmx.txt
$P -d $O/r8b_p8 -- python3 $R/bench.py --steps 20 --warmup 2 --no-secondary --model llama3-8b --ftype Q4_K_M --mb-size 1 > $O/r8b_p8.log 2>&1 || { tail -5 $O/r8b_p8.log; exit 1; }
python3 $R/tools/prof_summary.py $O/r8b_p8 > $O/r8b_p8.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/r8b_pmc -o run -- python3 $R/tools/gemv_bench.py --M 256 --iters 5 --gemm 4 --shapes 70b.gateup > $O/r8b_pmc.log 2>&1 || { tail -5 $O/r8b_pmc.log; exit 1; }
python3 $R/tools/pmc_summary.py $O/r8b_pmc > $O/r8b_pmc.txt; cat $O/r8b_pmc.txt | cut -c1-400
