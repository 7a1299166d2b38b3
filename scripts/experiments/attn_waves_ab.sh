#!/bin/bash
# decode attention 4 vs 8 waves per workgroup: engine tests, then 70B mb64 / mb1 and 8B mb1 benches (2 reps),
# then the kernel's own time from rocprofv3 at 70B mb64
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "attn or attention or engine or pipeline or spec" > $O/aw_tests.log 2>&1 || { tail -30 $O/aw_tests.log; exit 1; }
tail -1 $O/aw_tests.log
for rep in 1 2; do
for w in 4 8; do
  for a in "--mb-size 64" "--mb-size 1" "--model llama3-8b --ftype Q4_K_M --mb-size 1"; do
    MIPIPE_ATTN_WAVES=$w timeout -k 10 300 python3 bench.py $a --steps 20 --warmup 3 > $O/aw.log 2>&1 || { tail -5 $O/aw.log; exit 1; }
    echo "waves=$w $a: $(grep -o '"value": [0-9.]*' $O/aw.log)"
  done
done
done
cd /tmp
for w in 4 8; do
  export MIPIPE_ATTN_WAVES=$w
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/aw_prof_$w -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 > $O/aw_prof_$w.log 2>&1 || { tail -5 $O/aw_prof_$w.log; exit 1; }
  echo "== waves=$w"; python3 $R/tools/prof_summary.py $O/aw_prof_$w | sed -n '/last 5 decode/,$p' | grep -i "attn\|last 5"
done
