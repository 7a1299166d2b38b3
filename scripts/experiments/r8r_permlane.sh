#!/bin/bash
# r8r: decode attention column reductions on v_permlane16/32_swap instead of ds_bpermute: oracle tests, 70B mb256 at 128 / 2K contexts, 8B mb1
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 400 python -u -m pytest -q --timeout 250 --timeout-method thread -m gpu -p no:cacheprovider"
$T tests/test_attn_wave_gpu.py tests/test_engine_gpu.py -k "attn or wave or decode or reference or fp8 or single or 70b_width" > $O/r8r_t0.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" $O/r8r_t0.log | tail -4; [ $rc -gt 1 ] && exit $rc

cd /tmp
P="timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run"
pr() { local n=$1; shift; $P -d $O/r8r_$n -- python3 $R/bench.py --no-secondary "$@" > $O/r8r_$n.log 2>&1 || { tail -3 $O/r8r_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r8r_$n > $O/r8r_$n.txt; rm -rf $O/r8r_$n
  echo "== $n $(grep -o '"value": [0-9.]*' $O/r8r_$n.log) $(grep -m2 -E 'attn_decode' $O/r8r_$n.txt | tail -1 | cut -c1-100)"; }
pr 70b_al0 --steps 6 --warmup 2

pr 8b1 --steps 20 --warmup 2 --model llama3-8b --ftype Q4_K_M --mb-size 1
pr 70b_2k_al0 --steps 4 --warmup 1 --prompt-len 1984

