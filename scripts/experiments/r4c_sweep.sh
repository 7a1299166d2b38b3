#!/bin/bash
# gemvs plan sweep on 8B Q4_K_M mb1 (S = super-blocks per wave target, MINWG = min workgroups)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 200 python -u -m pytest tests/test_gemvs_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/r4c_tests.log 2>&1 || { tail -5 $O/r4c_tests.log; exit 1; }
tail -1 $O/r4c_tests.log
b() { timeout -k 10 120 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 40 --warmup 5 "$@" > $O/r4c_b.log 2>&1 || { tail -3 $O/r4c_b.log; exit 1; }; grep -o '"value": [0-9.]*' $O/r4c_b.log; }
echo -n "old path: "; b --set small_gemv=false
for s in 4 8 16; do for w in 256 512; do
  echo -n "S=$s MINWG=$w: "; MIPIPE_GEMVS_S=$s MIPIPE_GEMVS_MINWG=$w b
done; done
