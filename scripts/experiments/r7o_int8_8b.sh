#!/bin/bash
# why 8B mb256 shows no int8_gemm gain: engine log + kernel profile of the int8 round
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_i8b -o run --output-format csv -- \
  python3 $R/bench.py --model llama3-8b --ftype Q4_K_M --steps 8 --warmup 2 --no-secondary --set int8_gemm=true > $O/prof_i8b.log 2>&1 || { tail -5 $O/prof_i8b.log; exit 1; }
grep -E "int8_gemm|value" $O/prof_i8b.log | cut -c1-160
PROF_SEQ=0 python3 $R/tools/prof_summary.py $O/prof_i8b > $O/prof_8b_mb256_int8.txt && tail -14 $O/prof_8b_mb256_int8.txt
rm -rf $O/prof_i8b
