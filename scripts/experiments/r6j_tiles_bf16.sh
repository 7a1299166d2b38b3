#!/bin/bash
# gemm3 tile shapes for the split-K shapes; bf16 8B (native bf16 MFMA) single stream / mb64; 8B gate/up hot vs cold
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u tools/gemv_bench.py --gemm 3 --M 256 --iters 20 --shapes 70b.qkv,70b.o,70b.down,8b.down \
  --g3 "256,128,0;128,256,0;128,256,8;128,128,0;256,256,16" > $O/r6j_g3tiles.log 2>&1 || { tail -5 $O/r6j_g3tiles.log; exit 1; }
grep -h '"us"' $O/r6j_g3tiles.log | cut -c1-170
timeout -k 10 200 python -u tools/gemv_bench.py --M 1 --iters 50 --shapes 8b.gateup,8b.o --types Q4_K --copies 1 > $O/r6j_hot.log 2>&1 \
  && timeout -k 10 200 python -u tools/gemv_bench.py --M 1 --iters 50 --shapes 8b.gateup,8b.o --types Q4_K > $O/r6j_cold.log 2>&1 \
  || { tail -5 $O/r6j_cold.log; exit 1; }
grep -h '"us"' $O/r6j_hot.log $O/r6j_cold.log | cut -c1-150
for mb in 1 64; do
  timeout -k 10 300 python bench.py --model llama3-8b --ftype BF16 --mb-size $mb --steps 20 --warmup 3 --no-secondary \
    > $O/r6j_bf16_mb$mb.log 2>&1 || { tail -5 $O/r6j_bf16_mb$mb.log; exit 1; }
  echo "bf16 mb$mb $(grep -o '"value": [0-9.]*' $O/r6j_bf16_mb$mb.log)"
done
timeout -k 10 300 python -u tools/torch_mm_probe.py --M 256,512 > $O/r6j_torch_mm.log 2>&1 || { tail -5 $O/r6j_torch_mm.log; exit 1; }
cat $O/r6j_torch_mm.log
for v in 0 2 3 0; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-secondary --set prefill_gemm_v=$v > $O/r6j_bench_v$v.log 2>&1 \
    || { tail -5 $O/r6j_bench_v$v.log; exit 1; }
  echo "gemm_v=$v $(grep -o '"value": [0-9.]*' $O/r6j_bench_v$v.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r6j_prof_auto -o run -- python bench.py --steps 10 --warmup 2 \
  --no-secondary > $O/r6j_prof_auto.log 2>&1 || { tail -5 $O/r6j_prof_auto.log; exit 1; }
python tools/prof_db_summary.py $O/r6j_prof_auto 5 > $O/r6j_prof_auto.txt && rm -rf $O/r6j_prof_auto
head -12 $O/r6j_prof_auto.txt
