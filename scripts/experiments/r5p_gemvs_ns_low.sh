#!/bin/bash
# gemvs ring depth 2 / 3 (more resident workgroups) vs 4, single stream
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 env MIPIPE_GEMVS_NS=2 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gemvs_gpu.py > $O/r5p_tests.log 2>&1 || { tail -20 $O/r5p_tests.log; exit 1; }
tail -1 $O/r5p_tests.log
for ns in 0 2 3 0 2 3; do
  MIPIPE_GEMVS_NS=$ns timeout -k 10 300 python bench.py --mb-size 1 --steps 20 --warmup 3 > $O/r5p.log 2>&1 || { tail -5 $O/r5p.log; exit 1; }
  echo "ns=$ns 70b mb1 $(grep -o '"value": [0-9.]*' $O/r5p.log)"
  MIPIPE_GEMVS_NS=$ns timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 40 --warmup 3 > $O/r5p.log 2>&1 || { tail -5 $O/r5p.log; exit 1; }
  echo "ns=$ns 8b mb1 $(grep -o '"value": [0-9.]*' $O/r5p.log)"
done
