#!/bin/bash
# which decode-attention variant runs with MIPIPE_ATTN_PF_MAXWG=0 at mb256, and its time
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
for v in 1073741824 0; do
  MIPIPE_ATTN_PF_MAXWG=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pn_$v -o run --output-format csv -- \
    python3 $R/bench.py --steps 6 --warmup 1 --no-secondary > $O/pn.log 2>&1 || { tail -5 $O/pn.log; exit 1; }
  echo "pf_maxwg=$v: $(grep -o '"value": [0-9.]*' $O/pn.log)"
  python3 $R/tools/prof_summary.py $O/pn_$v | grep attn_decode | head -3 | cut -c1-110
  rm -rf $O/pn_$v
done
