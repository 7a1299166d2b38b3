#!/bin/bash
# r8u: fused single-stream attention + o-projection (attn_o_max_ctx) on the round-4 attention body:
# tests, 8B / 70B mb1 A/B (kernels per token from the trace)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 400 python -u -m pytest -q --timeout 250 --timeout-method thread -m gpu -p no:cacheprovider"
$T tests/test_engine_gpu.py -k "attn_o or fused" > $O/r8u_t.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" $O/r8u_t.log | tail -3; [ $rc -gt 1 ] && exit $rc
BB="timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --no-secondary --mb-size 1"
for rep in 1 2; do for a in 0 256; do
  $BB --model llama3-8b --ftype Q4_K_M --set attn_o_max_ctx=$a > $O/r8u_8_$a.log 2>&1 || exit 1
  echo "8b mb1 attn_o_max_ctx=$a $(grep -o '"value": [0-9.]*' $O/r8u_8_$a.log)"
done; done
for a in 0 256; do $BB --set attn_o_max_ctx=$a > $O/r8u_70_$a.log 2>&1 || exit 1; echo "70b mb1 attn_o_max_ctx=$a $(grep -o '"value": [0-9.]*' $O/r8u_70_$a.log)"; done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r8u_p -- python3 $R/bench.py --steps 20 --warmup 2 --no-secondary --model llama3-8b --ftype Q4_K_M --mb-size 1 --set attn_o_max_ctx=256 > $O/r8u_p.log 2>&1 || exit 1
python3 $R/tools/prof_summary.py $O/r8u_p > $O/r8u_p.txt; rm -rf $O/r8u_p; sed -n '/last 5 decode/,/dispatch order/p' $O/r8u_p.txt | head -8
