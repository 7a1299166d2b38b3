#!/bin/bash
# r8d: single-stream (8B mb1) decode attention: context-length sweep and kernel-variant A/B (kernel traces)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
P="timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -o run"
B="python3 $R/bench.py --steps 20 --warmup 2 --no-secondary --model llama3-8b --ftype Q4_K_M --mb-size 1"
run() {  # name (env and EXTRA bench args set by the caller)
  local n=$1
  $P -d $O/r8d_$n -- $B $EXTRA > $O/r8d_$n.log 2>&1 || { tail -5 $O/r8d_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r8d_$n > $O/r8d_$n.txt
  echo "$n $(grep -o '"value": [0-9.]*' $O/r8d_$n.log) $(grep -m3 -E 'attn_decode|attn_o' $O/r8d_$n.txt | tail -1 | cut -c1-110)"
}
EXTRA="--prompt-len 8" run ctx8
EXTRA="--prompt-len 128" run ctx128
EXTRA="--prompt-len 1000" run ctx1000
export MIPIPE_ATTN_WAVE=1; EXTRA="--prompt-len 128" run wave128; unset MIPIPE_ATTN_WAVE
export MIPIPE_ATTN_PF_MAXWG=0; EXTRA="--prompt-len 128" run np128; unset MIPIPE_ATTN_PF_MAXWG
