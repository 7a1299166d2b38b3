#!/bin/bash
# prompt processing (64 x 512-token prompts, chunk 2048): exact f16 GEMMs vs int8_gemm, 70B and 8B
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
cat > /tmp/pp.py <<'PY'
import json, sys
sys.path.insert(0, sys.argv[1])
import bench
from mipipe.engine import Engine
model, ftype, i8 = sys.argv[2], sys.argv[3], sys.argv[4] == "1"
cfg = dict(synthetic=bench.MODELS[model], ftype=ftype, n_mb=1, mb_size=64, max_ctx=640, prefill_chunk=2048,
           int8_gemm=i8, seed=1)
with Engine(**cfg) as eng:
    r = eng.bench(prompt_len=512, warmup=1, steps=3)
print(json.dumps({"model": model, "int8_gemm": i8, "prompt_tok_s": round(r["prompt_tok_s"], 1),
                  "prefill_ms": round(r["prefill_ms"], 1)}), flush=True)
PY
for m in "llama3-70b Q4_K" "llama3-8b Q4_K_M"; do
  for i8 in 0 1; do
    timeout -k 10 300 python3 /tmp/pp.py $R $m $i8 2> $O/pp.err | tail -1 || { tail -5 $O/pp.err; exit 1; }
  done
done
