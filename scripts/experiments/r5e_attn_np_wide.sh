#!/bin/bash
# decode attention variant at wide micro-batches: prefetch (2 WG/CU) vs no-prefetch (3 WG/CU)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for mx in 1073741824 0; do
  for mb in 256 512; do
    MIPIPE_ATTN_PF_MAXWG=$mx timeout -k 10 300 python bench.py --steps 10 --warmup 2 --mb-size $mb > $O/r5e_$mx_$mb.log 2>&1 || { tail -5 $O/r5e_$mx_$mb.log; exit 1; }
    echo "pf_maxwg=$mx 70b mb$mb $(grep -o '"value": [0-9.]*' $O/r5e_$mx_$mb.log)"
  done
  MIPIPE_ATTN_PF_MAXWG=$mx timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --steps 10 --warmup 2 --mb-size 256 > $O/r5e_8b_$mx.log 2>&1 || { tail -5 $O/r5e_8b_$mx.log; exit 1; }
  echo "pf_maxwg=$mx 8b mb256 $(grep -o '"value": [0-9.]*' $O/r5e_8b_$mx.log)"
done
