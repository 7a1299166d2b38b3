#!/bin/bash
# r10ad: knob re-sweep on the current build -- 8B Q4_K_M single stream (gemvs knobs), 70B mb64 (decode GEMV knobs)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
b8() { timeout -k 10 200 env "$@" python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 32 --warmup 4 --no-secondary > $O/r10ad.log 2>&1 || { tail -3 $O/r10ad.log; exit 1; }; echo "8b mb1 $* $(grep -o '"value": [0-9.]*' $O/r10ad.log)"; }
b70() { timeout -k 10 200 env "$@" python bench.py --mb-size 64 --steps 8 --warmup 2 --no-secondary > $O/r10ad.log 2>&1 || { tail -3 $O/r10ad.log; exit 1; }; echo "70b mb64 $* $(grep -o '"value": [0-9.]*' $O/r10ad.log)"; }
b8 X=0
for v in 3 4; do b8 MIPIPE_GEMVS_NS=$v; done
for v in 32 48 96 128; do b8 MIPIPE_GEMVS_S=$v; done
for v in 128 384 512; do b8 MIPIPE_GEMVS_MINWG=$v; done
b8 X=0
b70 X=0
for v in 1 2; do b70 MIPIPE_GEMV2_TW=$v; done
b70 MIPIPE_GEMV_NW=4
for v in 64 256; do b70 MIPIPE_GEMM2_SPLIT_WG=$v; done
b70 X=0
