#!/bin/bash
# A/B of the GEMV x-ring option: timing sweep + SQ counters on the 70B gate/up shape.
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/pmc; mkdir -p $O
cd $R
for XR in 0 1; do
  MIPIPE_GEMV_XR=$XR timeout -k 10 300 python tools/gemv_bench.py --types Q4_K --M 1,16 --tpw 1,2,4 > $O/time_xr$XR.log 2>&1 || { tail -3 $O/time_xr$XR.log; exit 1; }
done
paste <(grep shape $O/time_xr0.log | cut -c1-110) <(grep shape $O/time_xr1.log | sed -E 's/.*"us": ([0-9.]+).*/xr1 \1/')
cd /tmp
for XR in 0 1; do
  MIPIPE_GEMV_XR=$XR timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD --kernel-include-regex gemv -d $O/xr$XR -o run --output-format csv -- python3 $R/tools/gemv_bench.py --shapes 70b.gateup --types Q4_K --M 1,16 --tpw 1,4 --iters 6 > $O/pmc_xr$XR.log 2>&1 || { tail -5 $O/pmc_xr$XR.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $O/xr0 $O/xr1
