#!/bin/bash
# decode attention at 70B mb256: timing probes without the global V / K append (results wrong, time only)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
for v in 0 1 2 3 0; do
  MIPIPE_ATTN_PROBE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pr_$v -o run --output-format csv -- \
    python3 $R/bench.py --steps 6 --warmup 1 --no-secondary > $O/pr.log 2>&1 || { tail -5 $O/pr.log; exit 1; }
  echo "probe=$v: $(python3 $R/tools/prof_summary.py $O/pr_$v | grep -m1 'us/round.*attn_decode' | cut -c1-100)"
  rm -rf $O/pr_$v
done
