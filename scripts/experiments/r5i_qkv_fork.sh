#!/bin/bash
# q|k|v side-stream fork for mixed-type layers (Q4_K_M): tests, then 8B single-stream A/B
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gemvs_gpu.py tests/test_engine_gpu.py > $O/r5i_tests.log 2>&1 || { tail -30 $O/r5i_tests.log; exit 1; }
tail -2 $O/r5i_tests.log
for f in 1 0 1 0; do
  MIPIPE_QKV_FORK=$f timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 40 --warmup 3 > $O/r5i_$f.log 2>&1 || { tail -5 $O/r5i_$f.log; exit 1; }
  echo "fork=$f 8b mb1 $(grep -o '"value": [0-9.]*' $O/r5i_$f.log)"
done
