#!/bin/bash
# r8o: exp2-domain lazy-rescale softmax in the decode attention: attention / engine oracle tests, kernel traces
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 500 python -u -m pytest -q --timeout 250 --timeout-method thread -m gpu -p no:cacheprovider"
$T tests/test_attn_wave_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_deterministic_gpu.py -k "attn or wave or decode or reference or fp8 or single or long or split or determin" > $O/r8o_t.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" $O/r8o_t.log | tail -8; [ $rc -gt 1 ] && exit $rc
cd /tmp
P="timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run"
pr() { local n=$1; shift; $P -d $O/r8o_$n -- python3 $R/bench.py --no-secondary "$@" > $O/r8o_$n.log 2>&1 || { tail -3 $O/r8o_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r8o_$n > $O/r8o_$n.txt; rm -rf $O/r8o_$n
  echo "== $n $(grep -o '"value": [0-9.]*' $O/r8o_$n.log) $(grep -m2 -E 'attn_decode' $O/r8o_$n.txt | tail -1 | cut -c1-100)"; }
pr 70b --steps 6 --warmup 2
pr 8b1 --steps 20 --warmup 2 --model llama3-8b --ftype Q4_K_M --mb-size 1
pr 70b_2k --steps 4 --warmup 1 --prompt-len 1984
