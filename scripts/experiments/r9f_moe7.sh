#!/bin/bash
# r9f: gemm4 MoE mode with 7-wave workgroups (224 columns) when the expert tiles then fill whole
# rounds over the 256 CUs (Mixtral gate/up: 1024 workgroups instead of 896): tests, then Mixtral A/B
# against 8 waves (knob GEMM4_NW=8), same library
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 600 python -u -m pytest -q --timeout 250 --timeout-method thread -m gpu -p no:cacheprovider"
$T tests/test_moe_gemm_gpu.py tests/test_gemm4_gpu.py > $O/r9f_t.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" $O/r9f_t.log | tail -4; [ $rc -ne 0 ] && exit $rc
$T tests/test_engine_gpu.py -k "moe or mixtral" > $O/r9f_t2.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" $O/r9f_t2.log | tail -4; [ $rc -ne 0 ] && exit $rc
BB="timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-secondary --model mixtral-8x7b --ftype Q4_K_M"
for rep in 1 2; do for nw in 0 8; do
  MIPIPE_GEMM4_NW=$nw $BB > $O/r9f_mx_$nw.log 2>&1 || { tail -3 $O/r9f_mx_$nw.log; exit 1; }
  echo "rep $rep GEMM4_NW=$nw (0 = auto): mixtral mb256 $(grep -o '"value": [0-9.]*' $O/r9f_mx_$nw.log)"
done; done
$BB --mb-size 64 > $O/r9f_mx64.log 2>&1 || exit 1; echo "mixtral mb64 $(grep -o '"value": [0-9.]*' $O/r9f_mx64.log)"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r9f_p -- python3 $R/bench.py --steps 10 --warmup 2 --no-secondary --model mixtral-8x7b --ftype Q4_K_M > $O/r9f_p.log 2>&1 || exit 1
python3 $R/tools/prof_summary.py $O/r9f_p > $O/r9f_p.txt; rm -rf $O/r9f_p; sed -n '/last 5 decode/,/dispatch order/p' $O/r9f_p.txt | head -8
