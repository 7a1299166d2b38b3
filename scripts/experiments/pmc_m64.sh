#!/bin/bash
# PMC passes on the 70B gate/up GEMV at M=64 (TW=1 vs TW=2): issue / wait / pipe counters
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/pmc_list.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" $O/pmc_list.txt | sort -u | tr '\n' ' ' | head -c 6000; echo
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM"
for tw in 1 2; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    MIPIPE_GEMV2_TW=$tw timeout -s KILL 90 rocprofv3 --pmc $P -d $O/pmc64_${tw}_$i -o run --output-format csv -- python3 $R/tools/gemv_bench.py --shapes 70b.gateup --M 64 --tpw 1 --iters 4 > $O/pmc64_${tw}_$i.log 2>&1 || { echo "pass $tw/$i failed"; tail -3 $O/pmc64_${tw}_$i.log; }
    python3 $R/tools/pmc_summary.py $O/pmc64_${tw}_$i | grep -A2 gemv2 | head -3
  done
done
