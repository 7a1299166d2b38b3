#!/bin/bash
# r9j: MoE down projection unsplit at 128-row expert tiles (r9i): Mixtral A/B against the old 2 splits
# (GEMM3_SPLIT=2), then the end-of-round check again on this final library: full GPU suite, smoke(),
# the driver's default bench line
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -q --timeout 250 --timeout-method thread -m gpu -p no:cacheprovider tests/test_moe_gemm_gpu.py > $O/r9j_t0.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" $O/r9j_t0.log | tail -3; [ $rc -ne 0 ] && exit $rc
BB="timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-secondary --model mixtral-8x7b --ftype Q4_K_M"
for rep in 1 2; do for sp in 0 2; do
  MIPIPE_GEMM3_SPLIT=$sp $BB > $O/r9j_mx.log 2>&1 || { tail -3 $O/r9j_mx.log; exit 1; }
  echo "rep $rep GEMM3_SPLIT=$sp (0 = new default, unsplit): mixtral mb256 $(grep -o '"value": [0-9.]*' $O/r9j_mx.log)"
done; done
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/r9j_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" $O/r9j_tests.log | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r9j_smoke.log 2>&1 || { tail -5 $O/r9j_smoke.log; exit 1; }
tail -1 $O/r9j_smoke.log
t0=$(date +%s); timeout -k 10 900 python3 bench.py > $O/r9j_bench.log 2>&1 || { tail -5 $O/r9j_bench.log; exit 1; }; echo "bench wall $(( $(date +%s) - t0 )) s"
tail -1 $O/r9j_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step']); [print(k, v) for k,v in d.get('secondary',{}).items()]"
