#!/bin/bash
# r12h: rpc workers on HIP stages, the CLI multi-process tests; the driver's bench line (all secondaries)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_api.py -m gpu \
  "tests/test_engine_gpu.py::test_multiprocess_pipeline_one_gpu_tcp" > $O/r12h_tests.log 2>&1; rc=$?; tail -6 $O/r12h_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/r12h_bench.log 2>&1; rc=$?; tail -2 $O/r12h_bench.log; exit $rc
