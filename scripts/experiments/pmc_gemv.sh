#!/bin/bash
# gemv2 row-group timings + one PMC pass (LDS / wait counters) on 70B gate/up
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemv or gemm" > $O/kt.log 2>&1 || { tail -30 $O/kt.log; exit 1; }
tail -1 $O/kt.log; cd /tmp
timeout -k 10 240 python3 $R/tools/gemv_bench.py --shapes 70b.qkv,70b.o,70b.gateup,70b.down --M 16,32,48,64 --tpw 1 > $O/gemv_mt.log 2>&1 || { tail -5 $O/gemv_mt.log; exit 1; }
cat $O/gemv_mt.log | grep -v amdgpu.ids
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d $O/pmc_gemv -o run --output-format csv -- python3 $R/tools/gemv_bench.py --shapes 70b.gateup --M 16,64 --tpw 1 --iters 4 > $O/pmc_gemv.log 2>&1 || { tail -5 $O/pmc_gemv.log; exit 1; }
python3 $R/tools/pmc_summary.py $O/pmc_gemv | grep -A3 gemv2
