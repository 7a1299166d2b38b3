#!/bin/bash
# Fused single-stream attention + o-projection: oracle tests, then 8B Q4_K_M mb1 A/B (two-kernel vs fused)
# at the bench context (max_ctx 192) and at 2K-token prompts (fused off there by default; forced on to measure)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -q -x -k "attention_o or matches_reference or graph_equals" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_ao.log 2>&1; rc=$?
tail -3 $O/t_ao.log
[ $rc -ne 0 ] && exit $rc
for args in "" "--prompt-len 440" "--prompt-len 2000"; do
  for amc in 0 4096 0 4096; do
    timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 40 --warmup 3 --no-secondary $args \
      --set attn_o_max_ctx=$amc > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "8b mb1 [$args] attn_o_max_ctx=$amc $(grep -o '"value": [0-9.]*' $O/b.log) $(grep -o '"max_ctx": [0-9]*' $O/b.log)"
  done
done
