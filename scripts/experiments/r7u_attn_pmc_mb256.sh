#!/bin/bash
# PMC passes on the decode attention at 70B mb256, 128-token contexts (eager launches), counters on attn_decode only
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM"
P2="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"
P3="FETCH_SIZE TCC_HIT_sum"
P4="SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SMEM SQ_WAIT_INST_ANY"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-include-regex attn_decode -d $O/pmcw_$i -o run --output-format csv -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-secondary --no-graphs > $O/pmcw_$i.log 2>&1 \
    || { echo "pass $i failed"; tail -3 $O/pmcw_$i.log; exit 1; }
  python3 $R/tools/pmc_summary.py $O/pmcw_$i > $O/pmcw_$i.txt; grep -A3 attn_decode $O/pmcw_$i.txt | head -4
  rm -rf $O/pmcw_$i
done
