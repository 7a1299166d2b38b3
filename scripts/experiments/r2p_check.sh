#!/bin/bash
# full GPU suite + benches after failover / probe / spawn-cli / load work
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q -rs --timeout 120 --timeout-method thread > $O/r2p_tests.log 2>&1 || { tail -40 $O/r2p_tests.log; exit 1; }
tail -3 $O/r2p_tests.log
grep -A2 "test_gpu_device_probe" $O/r2p_tests.log | head -3
timeout -k 10 200 python bench.py > $O/r2p_bench70b_mb64.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 50 > $O/r2p_bench8b_mb1.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mb-size 1 --steps 20 > $O/r2p_bench70b_mb1.log 2>&1 || exit 1
python -c "
from mipipe.engine import device_probe; print(device_probe(0))" > $O/r2p_probe.log 2>&1 || exit 1
