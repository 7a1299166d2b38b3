#!/bin/bash
# PMC passes on the prompt GEMM v2 (70B gate/up, M=256): is it LDS-, MFMA- or issue-bound?
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $O/pmcg2_$i -o run --output-format csv -- python3 $R/tools/gemv_bench.py --gemm 2 --shapes 70b.gateup --M 256 --iters 4 > $O/pmcg2_$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/pmcg2_$i.log; exit 1; }
  python3 $R/tools/pmc_summary.py $O/pmcg2_$i > $O/pmcg2_$i.txt; grep -A3 gemv2 $O/pmcg2_$i.txt | head -4
done
