#!/bin/bash
# rocprofv3 kernel summaries of the other benchmark configs (8B mb64, 8B 32K-context single stream, 70B single stream)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ps_$name -o run --output-format csv -- python3 $R/bench.py "$@" > $O/ps_$name.log 2>&1 || { tail -5 $O/ps_$name.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/ps_$name > $O/prof_$name.txt
  echo "== $name: $(grep -o '"value": [0-9.]*' $O/ps_$name.log)"; sed -n '/last 5 decode/,$p' $O/prof_$name.txt | head -7
  rm -rf $O/ps_$name
}
run 8b_mb64 --model llama3-8b --ftype Q4_K_M --steps 10 --warmup 2
run 8b_ctx32k_mb1 --model llama3-8b --ftype Q4_K_M --mb-size 1 --prompt-len 32768 --steps 10 --warmup 2
run 70b_mb1 --mb-size 1 --steps 10 --warmup 2
