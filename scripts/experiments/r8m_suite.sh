#!/bin/bash
# r8m: the whole GPU test suite on the round-4 tree, then the PMC passes of r8l
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/r8m_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" $O/r8m_tests.log | tail -15
[ $rc -gt 1 ] && exit $rc
bash scripts/experiments/r8l_pmc.sh
exit $rc
