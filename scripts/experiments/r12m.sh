#!/bin/bash
# r12m (round-6 final build): full GPU suite, smoke, the driver's bench line; MoE down split-K A/B (GEMM3_SPLIT)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r12m_tests.log 2>&1; rc=$?; tail -3 $O/r12m_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r12m_smoke.log 2>&1; rc=$?; tail -1 $O/r12m_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/r12m_bench.log 2>&1; rc=$?; tail -1 $O/r12m_bench.log; [ $rc -ne 0 ] && exit $rc
run() { local n=$1 e="$2"; shift 2; timeout -k 10 300 env $e python3 -u $R/bench.py --no-secondary "$@" > $O/r12m_$n.log 2>&1 || { tail -5 $O/r12m_$n.log; exit 1; }
  echo "== $n $(grep -o '"value": [0-9.]*' $O/r12m_$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r12m_$n.log)"; }
for s in 0 2 4; do run mix_split$s "MIPIPE_GEMM3_SPLIT=$s" --model mixtral-8x7b --ftype Q4_K_M --mb-size 256; done
