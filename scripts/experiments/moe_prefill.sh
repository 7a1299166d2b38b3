#!/bin/bash
# Mixtral prompt processing: MoE v2 in 64-token slices vs v1 (MIPIPE_MOE_V=1), plus the MoE tests
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "moe or engine_matches or spec or prefill" > $O/moe_tests.log 2>&1 || { tail -30 $O/moe_tests.log; exit 1; }
tail -1 $O/moe_tests.log
cat > $O/mpf.py <<'PY'
import json, sys, torch
sys.path.insert(0, ".")
from mipipe.engine import Engine
import bench as B
torch.cuda.set_device(0)
e = Engine(synthetic=B.MODELS["mixtral-8x7b"], ftype="Q4_K_M", n_mb=1, mb_size=32, max_ctx=640, prefill_chunk=256,
           mode="local", stages=1, devices=[0])
r = e.bench(prompt_len=512, warmup=1, steps=4)
print(json.dumps(dict(prompt_tok_s=round(r["prompt_tok_s"], 1), prefill_ms=round(r["prefill_ms"], 1),
                      decode_tok_s=round(r["decode_tok_s"], 1))), flush=True)
PY
for v in 1 2; do
  MIPIPE_MOE_V=$v timeout -k 10 300 python3 $O/mpf.py > $O/mpf.log 2>&1 || { tail -5 $O/mpf.log; exit 1; }
  echo "moe v$v: $(grep '^{' $O/mpf.log)"
done
