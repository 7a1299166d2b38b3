#!/bin/bash
# r10al: hybrid CPU/GPU split speed (engine gpu_layers = llama-cli -ngl N): Llama-3-8B Q4_K_M single stream with the last
# N of 32 layers on the GPU, the rest on the CPU stage (16 host threads on this box)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
for n in 32 28 16; do
  timeout -k 10 400 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 6 --warmup 1 --no-secondary --set gpu_layers=$n --set threads=16 > $O/r10al_$n.log 2>&1 || { tail -5 $O/r10al_$n.log; exit 1; }
  echo "8b mb1 -ngl $n $(grep -o '"value": [0-9.]*' $O/r10al_$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r10al_$n.log)"
done
