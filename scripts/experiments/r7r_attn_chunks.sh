#!/bin/bash
# decode attention time at mb256 vs context length: 4 chunks of 32 keys (balanced over 4 waves) vs 5
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
for pl in 96 100 128 160; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pa_$pl -o run --output-format csv -- \
    python3 $R/bench.py --steps 6 --warmup 1 --no-secondary --prompt-len $pl > $O/pa.log 2>&1 || { tail -5 $O/pa.log; exit 1; }
  echo "prompt $pl: $(grep -o '"value": [0-9.]*' $O/pa.log) $(python3 $R/tools/prof_summary.py $O/pa_$pl | grep -m1 'attn_decode_kernel' | cut -c1-60)"
  rm -rf $O/pa_$pl
done
