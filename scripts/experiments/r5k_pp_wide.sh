#!/bin/bash
# emulated PP=2 (two stages on one GPU, LocalLink) with wide micro-batches: plumbing check at mb 256
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for mb in 64 256; do
  timeout -k 10 300 ./distributed-llm-pipeline_amd/bin/mi-cli --synthetic llama3-8b --ftype Q4_K_M --bench --mb-size $mb --micro-batches 3 --stages 2 --devices 0,0 -c 256 > $O/r5k_pp2_$mb.json 2> $O/r5k_pp2_$mb.log || { tail -5 $O/r5k_pp2_$mb.log; exit 1; }
  echo "pp2 emulated mb$mb x3: $(tail -c 330 $O/r5k_pp2_$mb.json)"
done
