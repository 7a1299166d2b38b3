#!/bin/bash
# r10d: 70B mb256 A/B -- split-K projections on gemm2 (auto) vs gemm4 (prefill_gemm_v=4, now free of
# the dead-read hazard and with saddr DMA), alternated; gemm4 gate/up PMC passes (compare r9b);
# kernel-trace profile of the default
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
for rep in 1 2; do
  for v in 0 4; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-secondary --set prefill_gemm_v=$v > $O/r10d_70b_v$v.log 2>&1 || { tail -5 $O/r10d_70b_v$v.log; exit 1; }
    echo "rep $rep 70b mb256 prefill_gemm_v=$v $(grep -o '"value": [0-9.]*' $O/r10d_70b_v$v.log)"
  done
done
timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --steps 10 --warmup 3 --no-secondary --set prefill_gemm_v=4 > $O/r10d_8b256_v4.log 2>&1 || exit 1
echo "8b mb256 prefill_gemm_v=4 $(grep -o '"value": [0-9.]*' $O/r10d_8b256_v4.log)"
timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --steps 10 --warmup 3 --no-secondary > $O/r10d_8b256_v0.log 2>&1 || exit 1
echo "8b mb256 auto $(grep -o '"value": [0-9.]*' $O/r10d_8b256_v0.log)"
B="python3 $R/tools/gemv_bench.py --M 256 --iters 5 --gemm 4 --shapes 70b.gateup"
pass() { local n=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $O/r10d_$n -o run -- $B > $O/r10d_$n.log 2>&1 || { tail -3 $O/r10d_$n.log; exit 1; }
  python3 $R/tools/pmc_summary.py $O/r10d_$n | grep -A2 gemm4 | cut -c1-600; rm -rf $O/r10d_$n; }
cd /tmp && export TMPDIR=/tmp
pass lds SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
pass mfma SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
cd $R
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r10d_p -- python3 $R/bench.py --steps 10 --warmup 3 --no-secondary > $O/r10d_prof.log 2>&1 || { tail -5 $O/r10d_prof.log; exit 1; }
grep -o '"value": [0-9.]*' $O/r10d_prof.log
python3 tools/prof_summary.py $O/r10d_p > $O/r10d_prof_summary.txt && head -30 $O/r10d_prof_summary.txt
rm -rf $O/r10d_p
