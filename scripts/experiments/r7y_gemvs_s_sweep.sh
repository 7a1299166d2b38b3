#!/bin/bash
# gemvs work target (super-blocks per wave) and workgroup floor for 8B Q4_K_M single stream
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for s in 64 32 16 64 128; do
  MIPIPE_GEMVS_S=$s timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 40 --warmup 3 --no-secondary > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "8b mb1 GEMVS_S=$s $(grep -o '"value": [0-9.]*' $O/b.log)"
done
for w in 512 1024; do
  MIPIPE_GEMVS_MINWG=$w timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 40 --warmup 3 --no-secondary > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "8b mb1 GEMVS_MINWG=$w $(grep -o '"value": [0-9.]*' $O/b.log)"
done
