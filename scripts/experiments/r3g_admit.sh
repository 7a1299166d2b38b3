#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for B in 64 16; do
  timeout -k 10 300 python3 tools/admit_probe.py --mb-size $B > $O/admit_$B.log 2>&1 || { tail -5 $O/admit_$B.log; exit 1; }
  tail -1 $O/admit_$B.log
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_admit -o run --output-format csv -- python3 $R/tools/admit_probe.py --mb-size 64 --rounds 10 > $O/prof_admit.log 2>&1 || { tail -5 $O/prof_admit.log; exit 1; }
python3 $R/tools/prof_summary.py $O/prof_admit | head -24
