#!/bin/bash
# gemvs2 at NS 2 and 6 waves/SIMD (5 VGPR spills) vs two separate launches, 8B Q4_K_M single stream
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gemvs_gpu.py > $O/r5q_tests.log 2>&1 || { tail -20 $O/r5q_tests.log; exit 1; }
tail -1 $O/r5q_tests.log
for f in 1 0 1 0; do
  MIPIPE_GEMVS2=$f timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 40 --warmup 3 > $O/r5q.log 2>&1 || { tail -5 $O/r5q.log; exit 1; }
  echo "gemvs2=$f 8b mb1 $(grep -o '"value": [0-9.]*' $O/r5q.log)"
done
