#!/bin/bash
# r10p: hybrid CPU/GPU split (-ngl N < n_layer) tests; MALL prefetch with graphs off (is the captured
# side branch serialized?); kernel summaries: 8B mb1 with the prefetch, 70B mb64 (the GEMV path)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_hybrid_gpu.py tests/test_prefetch_gpu.py > $O/r10p_t.log 2>&1 || { tail -40 $O/r10p_t.log; exit 1; }
grep -E "PASS|FAIL|SKIP|passed|failed" $O/r10p_t.log | tail -12
for v in 0 256; do
  MIPIPE_PREFETCH=$v timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 32 --warmup 4 --no-secondary --no-graphs > $O/r10p_8b_ng_$v.log 2>&1 || { tail -5 $O/r10p_8b_ng_$v.log; exit 1; }
  echo "8b mb1 no-graphs PREFETCH=$v $(grep -o '"value": [0-9.]*' $O/r10p_8b_ng_$v.log)"
done
cd /tmp && export TMPDIR=/tmp
prof() { local n=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r10p_$n -- python3 $R/bench.py --steps 10 --warmup 2 --no-secondary "$@" > $O/r10p_$n.log 2>&1 || { tail -3 $O/r10p_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r10p_$n > $O/r10p_prof_$n.txt; rm -rf $O/r10p_$n; echo "== $n $(grep -o '"value": [0-9.]*' $O/r10p_$n.log)"; sed -n '/last 5 decode/,/dispatch order/p' $O/r10p_prof_$n.txt | head -12; }
MIPIPE_PREFETCH=256 prof 8b_mb1_prefetch --model llama3-8b --ftype Q4_K_M --mb-size 1
prof 70b_mb64 --mb-size 64
