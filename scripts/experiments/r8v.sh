#!/bin/bash
# r8v: (1) 70B mb256 at 2K contexts with the fp8 KV cache (decode attention per layer from the
# kernel trace) against f16; (2) the 70B-width oracle with gemm4 split-K decode GEMMs, repeated
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 500 python3 -u scripts/experiments/r8v_oracle_v4.py > $O/r8v_o.log 2>&1 || { tail -5 $O/r8v_o.log; exit 1; }
grep -E "prefill_gemm_v|same tokens" $O/r8v_o.log
cd /tmp
for kv in fp8 f16; do
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $O/r8v_p_$kv -- python3 $R/bench.py --steps 6 --warmup 2 --no-secondary --prompt-len 1984 --set kv_dtype=$kv > $O/r8v_p_$kv.log 2>&1 || exit 1
python3 $R/tools/prof_summary.py $O/r8v_p_$kv > $O/r8v_p_$kv.txt; rm -rf $O/r8v_p_$kv
echo "== 2K kv=$kv $(grep -o '"value": [0-9.]*' $O/r8v_p_$kv.log) $(grep -m1 attn_decode $O/r8v_p_$kv.txt | sed -n 1p)"
sed -n '/last 5 decode/,/dispatch order/p' $O/r8v_p_$kv.txt | grep -m3 "attn\|wall"
done
