#!/bin/bash
# PMC passes on GEMM v3 (70B gate/up, M=256, 256x256 tiles): MFMA busy, VALU, LDS, waits
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM"
P3="GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $O/pmcg3_$i -o run --output-format csv -- python3 $R/tools/gemv_bench.py --gemm 3 --shapes 70b.gateup --M 256 --iters 4 > $O/pmcg3_$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/pmcg3_$i.log; exit 1; }
  python3 $R/tools/pmc_summary.py $O/pmcg3_$i > $O/pmcg3_$i.txt; grep -A3 gemm3 $O/pmcg3_$i.txt | head -4
done
