#!/bin/bash
# r10z: round-end check -- the whole GPU suite, smoke(), the default bench line (with secondaries)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/r10z_tests.log 2>&1; rc=$?
tail -3 $O/r10z_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r10z_smoke.log 2>&1 || { tail -5 $O/r10z_smoke.log; exit 1; }
tail -1 $O/r10z_smoke.log
