#!/bin/bash
# Full 1-GPU check: GPU tests -> benches (70B default mb256 + secondaries / mb16 / mb1, 8B mb1 / mb256, Mixtral mb256) -> mi-cli on GPU ->
# rocprofv3 kernel stats of the 70B bench.  Summaries land in gpurun_out/ (copied to profiles/).
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
step() { echo "== $1"; }
step tests
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" $O/tests.log | tail -12
[ $rc -gt 1 ] && exit $rc
step bench70b
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/b70.log 2>&1 || { tail -5 $O/b70.log; exit 1; }
grep '"value"' $O/b70.log | tee $O/bench_default.json
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --mb-size 16 > $O/b70_16.log 2>&1 || { tail -5 $O/b70_16.log; exit 1; }
grep '"value"' $O/b70_16.log | tee $O/bench_70b_mb16.json
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --mb-size 1 > $O/b70_1.log 2>&1 || { tail -5 $O/b70_1.log; exit 1; }
grep '"value"' $O/b70_1.log | tee $O/bench_70b_mb1.json
step bench8b
timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --steps 30 --warmup 3 --mb-size 1 > $O/b8.log 2>&1 || { tail -5 $O/b8.log; exit 1; }
grep '"value"' $O/b8.log | tee $O/bench_8b_mb1.json
timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --steps 30 --warmup 3 > $O/b8_64.log 2>&1 || { tail -5 $O/b8_64.log; exit 1; }
grep '"value"' $O/b8_64.log | tee $O/bench_8b_mb256.json
step mixtral
timeout -k 10 300 python bench.py --model mixtral-8x7b --ftype Q4_K_M --steps 20 --warmup 3 > $O/bmx.log 2>&1 || { tail -5 $O/bmx.log; exit 1; }
grep '"value"' $O/bmx.log | tee $O/bench_mixtral_mb256.json
step cli
timeout -k 10 300 ./distributed-llm-pipeline_amd/bin/mi-cli --synthetic llama3-8b --ftype Q4_K_M --bench --mb-size 4 --micro-batches 2 --stages 2 --devices 0,0 --trace $O/trace_8b_pp2.json > $O/cli_bench.json 2> $O/cli_bench.log || { tail -5 $O/cli_bench.log; exit 1; }
tail -c 400 $O/cli_bench.json
step prof
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-secondary > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
PROF_SEQ=0 python3 $R/tools/prof_summary.py $O/prof > $O/prof_bench_default.txt && head -30 $O/prof_bench_default.txt
