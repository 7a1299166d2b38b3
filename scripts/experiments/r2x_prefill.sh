#!/bin/bash
# prompt processing with GEMM v2 vs v1 (Engine.bench: 64 prompts x 512 tokens); GEMM tests
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k gemm > $O/r2x_tests.log 2>&1; rc=$?; tail -2 $O/r2x_tests.log; [ $rc = 0 ] || exit 1
cat > $O/pf2.py <<'PY'
import json, sys, torch
sys.path.insert(0, ".")
from mipipe.engine import Engine
import bench as B
model, ftype, v, chunk = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
torch.cuda.set_device(0)
e = Engine(synthetic=B.MODELS[model], ftype=ftype, n_mb=1, mb_size=64, max_ctx=640, prefill_chunk=chunk,
           prefill_gemm_v=v, mode="local", stages=1, devices=[0])
r = e.bench(prompt_len=512, warmup=1, steps=4)
print(json.dumps(dict(model=model, gemm_v=v, chunk=chunk, prompt_tok_s=round(r["prompt_tok_s"], 1),
                      prefill_ms=round(r["prefill_ms"], 1), decode_tok_s=round(r["decode_tok_s"], 1))), flush=True)
e.close()
PY
for m in "llama3-70b Q4_K" "llama3-8b Q4_K_M"; do
  for v in 2 1; do
    for c in 512 2048; do
      timeout -k 10 300 python3 $O/pf2.py $m $v $c >> $O/pf2.log 2>&1 || { tail -5 $O/pf2.log; exit 1; }
      tail -1 $O/pf2.log
    done
  done
done
