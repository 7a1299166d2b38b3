#!/bin/bash
# r10ab: Llama-3-8B BF16 at 64-row micro-batches: kernel summary of the engine, and per shape the GEMV (default at
# M <= 64) against gemm3 / gemm4 on 128-row tiles (cold weights)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
for g in 0 3 4; do
  timeout -k 10 200 python tools/gemv_bench.py --types BF16 --M 64 --iters 16 --gemm $g --shapes 8b.qkv,8b.o,8b.gateup,8b.down > $O/r10ab_g$g.log 2>&1 || { tail -5 $O/r10ab_g$g.log; exit 1; }
  echo "gemm $g"; grep -o '"shape": "[^"]*".*"us": [0-9.]*.*"GBps": [0-9.]*' $O/r10ab_g$g.log | sed 's/"type.*"us"/ us/'
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r10ab_p -- python3 $R/bench.py --model llama3-8b --ftype BF16 --mb-size 64 --steps 10 --warmup 2 --no-secondary > $O/r10ab_p.log 2>&1 || { tail -3 $O/r10ab_p.log; exit 1; }
python3 $R/tools/prof_summary.py $O/r10ab_p > $O/r10ab_prof.txt; rm -rf $O/r10ab_p
echo "== prof $(grep -o '"value": [0-9.]*' $O/r10ab_p.log)"; sed -n '/last 5 decode/,/dispatch order/p' $O/r10ab_prof.txt | head -12
