#!/bin/bash
# r11a: 8B Q4_K_M single stream, per-kernel times under knob variants of the small-M GEMV
# (ring depth, workgroup count / tiles per workgroup): which GEMV shapes are latency- vs balance-bound
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
prof() { local n=$1; shift; timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r11a_$n -- python3 $R/bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 30 --warmup 3 --no-secondary > $O/r11a_$n.log 2>&1 || { tail -3 $O/r11a_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r11a_$n > $O/r11a_prof_$n.txt; rm -rf $O/r11a_$n; echo "== $n $(grep -o '"value": [0-9.]*' $O/r11a_$n.log)"; sed -n '/last 5 decode/,/dispatch order/p' $O/r11a_prof_$n.txt | head -12; }
prof default
MIPIPE_GEMVS_NS=4 prof ns4
MIPIPE_GEMVS_NS=3 prof ns3
MIPIPE_GEMVS_MINWG=512 prof minwg512
MIPIPE_GEMVS_G=1 prof g1
MIPIPE_GEMVS_G=2 prof g2
MIPIPE_GEMVS_S=8 prof s8
