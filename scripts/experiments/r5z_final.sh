#!/bin/bash
# round-end check: GPU tests -> smoke -> driver bench command -> other configs -> rocprofv3 of the headline
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
echo "== tests"
timeout -k 10 700 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/r5z_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED" $O/r5z_tests.log | tail -8
[ $rc -gt 1 ] && exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r5z_smoke.log 2>&1 || { tail -5 $O/r5z_smoke.log; exit 1; }
tail -1 $O/r5z_smoke.log | cut -c1-200
echo "== bench"
b() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/r5z_$n.log 2>&1 || { tail -5 $O/r5z_$n.log; exit 1; }; grep '"value"' $O/r5z_$n.log > $O/r5z_$n.json; echo "$n $(grep -o '"value": [0-9.]*, "unit"[^}]*"ms_per_step": [0-9.]*' $O/r5z_$n.json)"; }
b default --gpus 1 --steps 20 --warmup 5
b 70b_mb512 --mb-size 512 --steps 10 --warmup 2
b 70b_mb64 --mb-size 64 --steps 20 --warmup 3
b 70b_mb1 --mb-size 1 --steps 20 --warmup 3
b 8b_mb1 --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 40 --warmup 3
b 8b_mb256 --model llama3-8b --ftype Q4_K_M --steps 20 --warmup 3
b mixtral_mb64 --model mixtral-8x7b --ftype Q4_K_M --mb-size 64 --steps 20 --warmup 3
echo "== prof"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r5z_prof -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 > $O/r5z_prof.log 2>&1 || { tail -5 $O/r5z_prof.log; exit 1; }
python3 $R/tools/prof_summary.py $O/r5z_prof > $O/r5z_prof_70b_mb256.txt && sed -n '/last 5/,$p' $O/r5z_prof_70b_mb256.txt | head -8
