#!/bin/bash
# r10b: the headline PP=8 launch rehearsed on ONE GPU (8 stage threads, 9 x 256 sequences, 72 graphs),
# f32 and bf16 stage boundaries, against PP=1 in the same call; tokens of both wires compared
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-secondary > $O/r10b_pp1.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' $O/r10b_pp1.log
timeout -k 10 700 python bench.py --gpus 8 --same-device --steps 10 --warmup 3 --no-secondary --dump-tokens $O/r10b_tok_f32.json > $O/r10b_pp8.log 2>&1 || { tail -5 $O/r10b_pp8.log; exit 1; }
grep -o '"value": [0-9.]*' $O/r10b_pp8.log
timeout -k 10 700 python bench.py --gpus 8 --same-device --steps 10 --warmup 3 --no-secondary --set act_dtype=bf16 --dump-tokens $O/r10b_tok_bf16.json > $O/r10b_pp8_bf16.log 2>&1 || { tail -5 $O/r10b_pp8_bf16.log; exit 1; }
grep -o '"value": [0-9.]*' $O/r10b_pp8_bf16.log
python - <<'PY'
import json
a = json.load(open("gpurun_out/r10b_tok_f32.json")); b = json.load(open("gpurun_out/r10b_tok_bf16.json"))
n = sum(len(x) for x in a); same = sum(1 for x, y in zip(a, b) for u, v in zip(x, y) if u == v)
seq_same = sum(1 for x, y in zip(a, b) if x == y)
print(json.dumps(dict(tokens=n, equal_tokens=same, frac=round(same / max(1, n), 4), seqs=len(a), equal_seqs=seq_same)))
PY
