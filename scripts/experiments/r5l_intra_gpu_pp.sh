#!/bin/bash
# intra-GPU pipelining: 2 stages on ONE GPU (own streams) with 2-3 micro-batches in flight vs 1 stage
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
run() { n=$1; shift; timeout -k 10 300 ./distributed-llm-pipeline_amd/bin/mi-cli --synthetic llama3-70b --ftype Q4_K --bench -c 192 "$@" > $O/r5l_$n.json 2> $O/r5l_$n.log || { tail -5 $O/r5l_$n.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/r5l_$n.json')); i=d.get('info',d); print('$n', 'ms_per_round=%.2f'%d['ms_per_round'], 'p50=%.2f'%d['p50_ms'])"; }
run s1_mb256 --mb-size 256 --micro-batches 1 --stages 1 --devices 0
run s2_mb256x2 --mb-size 256 --micro-batches 2 --stages 2 --devices 0,0
run s2_mb256x3 --mb-size 256 --micro-batches 3 --stages 2 --devices 0,0
run s2_mb128x3 --mb-size 128 --micro-batches 3 --stages 2 --devices 0,0
run s4_mb128x5 --mb-size 128 --micro-batches 5 --stages 4 --devices 0,0,0,0
