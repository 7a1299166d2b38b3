#!/bin/bash
# r10an: decode attention wave-kernel variants re-checked on the final build: inline-asm chunk loads with counted waits
# (ATTN_ASMLD=1), whole-line K loads (ATTN_KFL=1) vs default, 70B mb256 and mb64, alternated
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
b() { timeout -k 10 200 env "$@" python bench.py --steps 8 --warmup 2 --no-secondary $MB > $O/r10an.log 2>&1 || { tail -3 $O/r10an.log; exit 1; }; echo "$MB $* $(grep -o '"value": [0-9.]*' $O/r10an.log)"; }
for MB in "--mb-size 256" "--mb-size 64"; do
  for rep in 1 2; do b X=0; b MIPIPE_ATTN_ASMLD=1; b MIPIPE_ATTN_KFL=1; done
done
