#!/bin/bash
# Prompt processing (64 x 512-token prompts, chunk 2048) with / without gemm_splitk_store; 8B mb 64/128/256
# decode sweep (the round-2 GEMV->GEMM cliff); kernel profile of the 70B mb256 headline round
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cat > /tmp/pp.py <<'EOF'
import json, sys
sys.path.insert(0, sys.argv[1])
import bench
from mipipe.engine import Engine
model, ftype, sk = sys.argv[2], sys.argv[3], sys.argv[4] == "1"
cfg = dict(synthetic=bench.MODELS[model], ftype=ftype, n_mb=1, mb_size=64, max_ctx=640, prefill_chunk=2048,
           gemm_splitk_store=sk, seed=1)
with Engine(**cfg) as eng:
    r = eng.bench(prompt_len=512, warmup=1, steps=3)
print(json.dumps({"model": model, "splitk_store": sk, "prompt_tok_s": round(r["prompt_tok_s"], 1),
                  "prefill_ms": round(r["prefill_ms"], 1)}), flush=True)
EOF
for m in "llama3-70b Q4_K" "llama3-8b Q4_K_M"; do
  for sk in 0 1 0 1; do
    timeout -k 10 300 python3 /tmp/pp.py $R $m $sk 2> $O/pp.err | tail -1 || { tail -5 $O/pp.err; exit 1; }
  done
done
for mb in 64 128 256; do
  timeout -k 10 300 python3 $R/bench.py --model llama3-8b --ftype Q4_K_M --mb-size $mb --steps 15 --warmup 3 --no-secondary > $O/b8.log 2>&1 \
    || { tail -5 $O/b8.log; exit 1; }
  echo "8b mb$mb $(grep -o '"value": [0-9.]*' $O/b8.log) $(grep -o '"ms_per_step": [0-9.]*' $O/b8.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 $R/bench.py --steps 8 --warmup 2 --no-secondary > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
PROF_SEQ=0 python3 $R/tools/prof_summary.py $O/prof > $O/prof_70b_mb256.txt && tail -16 $O/prof_70b_mb256.txt
rm -rf $O/prof
