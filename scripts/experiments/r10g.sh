#!/bin/bash
# r10g: chained o -> gate/up -> down (GEMVS_CHAIN) -- oracle test, then 8B / 70B single-stream A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemvs_chain_gpu.py > $O/r10g_t.log 2>&1 || { tail -30 $O/r10g_t.log; exit 1; }
tail -2 $O/r10g_t.log
for rep in 1 2; do
  for c in 0 1; do
    MIPIPE_GEMVS_CHAIN=$c timeout -k 10 200 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 20 --warmup 5 --no-secondary > $O/r10g_8b_$c.log 2>&1 || { tail -5 $O/r10g_8b_$c.log; exit 1; }
    echo "rep $rep 8b mb1 GEMVS_CHAIN=$c $(grep -o '"value": [0-9.]*' $O/r10g_8b_$c.log)"
  done
done
for c in 0 1; do
  MIPIPE_GEMVS_CHAIN=$c timeout -k 10 300 python bench.py --mb-size 1 --steps 10 --warmup 3 --no-secondary > $O/r10g_70b_$c.log 2>&1 || { tail -5 $O/r10g_70b_$c.log; exit 1; }
  echo "70b mb1 GEMVS_CHAIN=$c $(grep -o '"value": [0-9.]*' $O/r10g_70b_$c.log)"
done
cd /tmp && export TMPDIR=/tmp && cd $R
MIPIPE_GEMVS_CHAIN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r10g_p -- python3 $R/bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 10 --warmup 3 --no-secondary > $O/r10g_prof.log 2>&1 || { tail -5 $O/r10g_prof.log; exit 1; }
python3 tools/prof_summary.py $O/r10g_p > $O/r10g_prof_summary.txt && sed -n '/last 5 decode rounds/,$p' $O/r10g_prof_summary.txt | head -14
rm -rf $O/r10g_p
