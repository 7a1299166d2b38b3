#!/bin/bash
# A/B two in-tree library builds on the same box: bench lines + decode kernel stats for each.
# usage: ab_lib.sh <libA.so> <libB.so> [bench args...]
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
A=$1; B=$2; shift 2
for rep in 1 2; do
for L in $A $B; do
  MIPIPE_LIB=$L timeout -k 10 200 python3 $R/bench.py "$@" > $O/ab_$L.log 2>&1 || { tail -5 $O/ab_$L.log; exit 1; }
  echo "$L: $(grep -o '"value": [0-9.]*' $O/ab_$L.log)"
done
done
for L in $A $B; do
  export MIPIPE_LIB=$L
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/ab_prof_$L -o run --output-format csv -- python3 $R/bench.py "$@" > $O/ab_prof_$L.log 2>&1 || { tail -5 $O/ab_prof_$L.log; exit 1; }
  echo "== $L"; python3 $R/tools/prof_summary.py $O/ab_prof_$L | sed -n '/last 5 decode/,$p' | head -8
done
