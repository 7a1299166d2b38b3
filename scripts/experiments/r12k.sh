#!/bin/bash
# r12k: MoE down split over K with the 96-row tiles (GEMM3_SPLIT forces it; it also forces the dense split-K shapes)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
run() { local n=$1 e="$2"; shift 2; timeout -k 10 300 env $e python3 -u $R/bench.py --no-secondary "$@" > $O/r12k_$n.log 2>&1 || { tail -5 $O/r12k_$n.log; exit 1; }
  echo "== $n $(grep -o '"value": [0-9.]*' $O/r12k_$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r12k_$n.log)"; }
for s in 0 2 3 4 0; do run mix_split$s "MIPIPE_GEMM3_SPLIT=$s" --model mixtral-8x7b --ftype Q4_K_M --mb-size 256; done
cd /tmp
export MIPIPE_GEMM3_SPLIT=2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r12k_prof -- python3 $R/bench.py --steps 30 --warmup 3 --no-secondary --model mixtral-8x7b --ftype Q4_K_M --mb-size 256 > $O/r12k_prof.log 2>&1 || { tail -3 $O/r12k_prof.log; exit 1; }
python3 $R/tools/prof_summary.py $O/r12k_prof > $O/r12k_prof_mixtral_split2.txt; rm -rf $O/r12k_prof; sed -n '/last 5 decode/,/dispatch order/p' $O/r12k_prof_mixtral_split2.txt | head -12
