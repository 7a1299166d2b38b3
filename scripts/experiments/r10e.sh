#!/bin/bash
# r10e: MoE gemm4 timing + PMC (is the Mixtral gate/up VALU-, latency- or issue-bound?), knob A/Bs;
# the scale.sh curve for BASELINE config 3 (8B bf16) rehearsed on one GPU
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
timeout -k 10 300 python tools/moe_bench.py --M 64,256 --knob GEMM4_WNT=0,2 > $O/r10e_moe.log 2>&1 || { tail -5 $O/r10e_moe.log; exit 1; }
cat $O/r10e_moe.log
B="python3 $R/tools/moe_bench.py --M 256 --phases gateup --iters 5"
pass() { local n=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $O/r10e_$n -o run -- $B > $O/r10e_$n.log 2>&1 || { tail -3 $O/r10e_$n.log; exit 1; }
  python3 $R/tools/pmc_summary.py $O/r10e_$n | grep -A2 gemm4 | cut -c1-600; rm -rf $O/r10e_$n; }
cd /tmp && export TMPDIR=/tmp
pass lds SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
pass mfma SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
cd $R
timeout -k 10 900 bash scripts/scale.sh --gpus 1,4 --same-device --steps 10 --warmup 3 -- --model llama3-8b --ftype BF16 --mb-size 64 > $O/r10e_scale_8b_bf16.json 2> $O/r10e_scale.err || { tail -5 $O/r10e_scale.err; exit 1; }
cat $O/r10e_scale_8b_bf16.json
