#!/bin/bash
# r8i: engine kernel traces, A/B: gemm4 LDS-DMA spread (70B mb256) and the MoE row tile (Mixtral mb256)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
P="timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -o run"
pr() { local n=$1; shift; $P -d $O/r8i_$n -- python3 $R/bench.py --steps 6 --warmup 2 --no-secondary "$@" > $O/r8i_$n.log 2>&1 || { tail -3 $O/r8i_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r8i_$n > $O/r8i_$n.txt; echo "== $n $(grep -o '"value": [0-9.]*' $O/r8i_$n.log)"; sed -n '/last 5 decode/,/dispatch order/p' $O/r8i_$n.txt | head -9 | cut -c1-120; }
export MIPIPE_GEMM4_SPREAD=0; pr 70sp0
export MIPIPE_GEMM4_SPREAD=2; pr 70sp2
unset MIPIPE_GEMM4_SPREAD
pr mx64 --model mixtral-8x7b --ftype Q4_K_M
export MIPIPE_GEMM3_BM=128; pr mx128 --model mixtral-8x7b --ftype Q4_K_M; unset MIPIPE_GEMM3_BM
# single-stream attention phase stamps (probe library, printf from block 0; graphs off so prints flush)
cd $R
MIPIPE_LIB=../lib_probes/libmipipe.so MIPIPE_ATTN_PROBE=4 timeout -k 10 200 python3 bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --no-secondary --steps 3 --warmup 1 --no-graphs > $O/r8i_stamps.log 2>&1 || { tail -3 $O/r8i_stamps.log; exit 1; }
grep "attn stamps" $O/r8i_stamps.log | head -6
# the driver's default bench line (all secondaries), timed
t0=$(date +%s); timeout -k 10 600 python3 bench.py > $O/r8i_bench.log 2>&1 || { tail -3 $O/r8i_bench.log; exit 1; }; echo "bench wall $(( $(date +%s) - t0 )) s"
tail -2 $O/r8i_bench.log | cut -c1-3000
