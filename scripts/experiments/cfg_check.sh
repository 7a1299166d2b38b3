#!/bin/bash
# BASELINE configs beyond the headline: 8B bf16 (PP=1 and PP=4 emulated on one GPU), Mixtral PP=4 emulated;
# 70B mb64 after the M > 32 split-K target change
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > $O/c70.log 2>&1 || { tail -5 $O/c70.log; exit 1; }
echo "70B mb64: $(grep -o '"value": [0-9.]*' $O/c70.log)"
for mb in 1 64; do
  timeout -k 10 300 python3 bench.py --model llama3-8b --ftype BF16 --mb-size $mb --steps 20 --warmup 3 > $O/c8bf_$mb.log 2>&1 || { tail -5 $O/c8bf_$mb.log; exit 1; }
  echo "8B bf16 mb$mb: $(grep -o '"value": [0-9.]*' $O/c8bf_$mb.log)"
done
B=./distributed-llm-pipeline_amd/bin/mi-cli
timeout -k 10 300 $B --synthetic llama3-8b --ftype BF16 --bench --mb-size 16 --micro-batches 4 --stages 4 --devices 0,0,0,0 --bench-steps 20 > $O/c8bf_pp4.json 2> $O/c8bf_pp4.log || { tail -5 $O/c8bf_pp4.log; exit 1; }
echo "8B bf16 PP4 emulated: $(tail -c 300 $O/c8bf_pp4.json)"
timeout -k 10 300 $B --synthetic mixtral-8x7b --ftype Q4_K_M --bench --mb-size 16 --micro-batches 4 --stages 4 --devices 0,0,0,0 --bench-steps 20 > $O/cmx_pp4.json 2> $O/cmx_pp4.log || { tail -5 $O/cmx_pp4.log; exit 1; }
echo "Mixtral PP4 emulated: $(tail -c 300 $O/cmx_pp4.json)"
