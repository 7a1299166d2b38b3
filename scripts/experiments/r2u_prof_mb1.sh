#!/bin/bash
# single-stream profiles (8B Q4_K_M, 70B Q4_K) with the current build
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
bash $R/scripts/experiments/prof_mb.sh u8b --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 30 || exit 1
bash $R/scripts/experiments/prof_mb.sh u70b --mb-size 1 --steps 20 || exit 1
