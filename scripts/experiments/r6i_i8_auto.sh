#!/bin/bash
# int8-activation GEMM prototype (tests + 70B shapes vs the f16 GEMMs), auto GEMM selection bench, long context
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_i8_gpu.py > $O/r6i_i8_tests.log 2>&1 || { tail -40 $O/r6i_i8_tests.log; exit 1; }
grep -E "NMSE|passed|failed" $O/r6i_i8_tests.log | tail -8
SH=70b.qkv,70b.o,70b.gateup,70b.down
for g in 8 3 2; do
  timeout -k 10 300 python -u tools/gemv_bench.py --gemm $g --M 256 --iters 20 --shapes $SH > $O/r6i_g$g.log 2>&1 \
    || { tail -5 $O/r6i_g$g.log; exit 1; }
  grep -h '"us"' $O/r6i_g$g.log | cut -c1-160
done
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > $O/r6i_bench_auto.log 2>&1 || { tail -5 $O/r6i_bench_auto.log; exit 1; }
cat $O/r6i_bench_auto.log | grep '"metric"' | cut -c1-400
grep -o '"secondary".*' $O/r6i_bench_auto.log
bash scripts/experiments/r6g_long_ctx.sh
