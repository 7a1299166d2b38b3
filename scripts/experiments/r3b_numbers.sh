#!/bin/bash
# round-2 numbers: full round check + long context
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
bash $R/scripts/round_check.sh || exit 1
cd $R && for cfg in "8192 1" "32768 1" "32768 8"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --model llama3-8b --ftype Q4_K_M --prompt-len $1 --mb-size $2 --steps 20 --warmup 2 > $O/lc.log 2>&1 || { tail -5 $O/lc.log; exit 1; }
  grep '"value"' $O/lc.log > $O/lc_$1_$2.json; echo "8B prompt $1 mb $2: $(grep -o '"value": [0-9.]*' $O/lc.log)"
done
