#!/bin/bash
# r8p: gemm4 for every wide GEMM (split-K shapes too, now with non-temporal weights) vs the auto choice;
# then the driver's default bench line with all secondaries
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
BB="timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-secondary"
$BB > $O/r8p_auto.log 2>&1 || { tail -3 $O/r8p_auto.log; exit 1; }
$BB --set prefill_gemm_v=4 > $O/r8p_v4.log 2>&1 || { tail -3 $O/r8p_v4.log; exit 1; }
$BB > $O/r8p_auto2.log 2>&1 || { tail -3 $O/r8p_auto2.log; exit 1; }
grep -H -o '"value": [0-9.]*' $O/r8p_*.log
t0=$(date +%s); timeout -k 10 600 python3 bench.py > $O/r8p_bench.log 2>&1 || { tail -3 $O/r8p_bench.log; exit 1; }; echo "bench wall $(( $(date +%s) - t0 )) s"
tail -1 $O/r8p_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step']); [print(k, v) for k,v in d.get('secondary',{}).items()]"
