#!/bin/bash
# First-pass GPU validation: kernel tests -> engine tests -> 1-GPU bench. Stops on crash/timeout.
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  tail -n 40 gpurun_out/$name.log
  return $rc
}
run kernels 420 python -m pytest tests/test_kernels_gpu.py -q -m gpu -p no:cacheprovider; rc=$?
[ $rc -gt 1 ] && exit $rc
run engine 420 python -m pytest tests/test_engine_gpu.py -q -m gpu -p no:cacheprovider; rc=$?
[ $rc -gt 1 ] && exit $rc
run bench 300 python bench.py --steps 10 --warmup 3
