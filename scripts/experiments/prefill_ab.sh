#!/bin/bash
# prefill (prompt processing) throughput: MFMA dequant-GEMM (prefill_gemm=true) vs the decode GEMV run over
# 64-row slices (prefill_gemm=false); 70B Q4_K and 8B Q4_K_M, 64 prompts x 512 tokens, chunk 256 / 512
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
cat > $O/pf.py <<'PY'
import json, sys, torch
sys.path.insert(0, ".")
from mipipe.engine import Engine
import bench as B
model, ftype, pg, chunk = sys.argv[1], sys.argv[2], sys.argv[3] == "1", int(sys.argv[4])
torch.cuda.set_device(0)
e = Engine(synthetic=B.MODELS[model], ftype=ftype, n_mb=1, mb_size=64, max_ctx=640, prefill_chunk=chunk,
           prefill_gemm=pg, mode="local", stages=1, devices=[0])
r = e.bench(prompt_len=512, warmup=1, steps=4)
print(json.dumps(dict(model=model, prefill_gemm=pg, chunk=chunk, prompt_tok_s=round(r["prompt_tok_s"], 1),
                      prefill_ms=round(r["prefill_ms"], 1), decode_tok_s=round(r["decode_tok_s"], 1))), flush=True)
e.close()
PY
for m in "llama3-70b Q4_K" "llama3-8b Q4_K_M"; do
  for pg in 1 0; do
    for ch in 256 512; do
      timeout -k 10 300 python3 $O/pf.py $m $pg $ch > $O/pf.log 2>&1 || { tail -5 $O/pf.log; exit 1; }
      grep '^{' $O/pf.log
    done
  done
done
