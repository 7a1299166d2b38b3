#!/bin/bash
# PMC passes on the decode attention at 2K contexts (70B mb64, eager launches), counters on attn_decode only
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM"
P2="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"
P3="FETCH_SIZE TCC_HIT_sum"

i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-include-regex attn_decode -d $O/pmca_$i -o run --output-format csv -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-secondary --no-graphs --prompt-len 2040 --mb-size 64 > $O/pmca_$i.log 2>&1 \
    || { echo "pass $i failed"; tail -3 $O/pmca_$i.log; exit 1; }
  python3 $R/tools/pmc_summary.py $O/pmca_$i > $O/pmca_$i.txt; grep -A3 attn_decode $O/pmca_$i.txt | head -4
  rm -rf $O/pmca_$i
done
