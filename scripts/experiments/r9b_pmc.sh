#!/bin/bash
# r9b: PMC passes on gemm4 gate/up (70B, M = 256) after the round-4 scalar-overhead cuts (compare r8l)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
B="python3 $R/tools/gemv_bench.py --M 256 --iters 5 --gemm 4 --shapes 70b.gateup"
pass() { local n=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $O/r9b_$n -o run -- $B > $O/r9b_$n.log 2>&1 || { tail -3 $O/r9b_$n.log; exit 1; }
  python3 $R/tools/pmc_summary.py $O/r9b_$n | grep -A2 gemm4 | cut -c1-600; rm -rf $O/r9b_$n; }
pass lds SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
pass mfma SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
