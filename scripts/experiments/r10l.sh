#!/bin/bash
# r10l: r10g (chain) + r10k (gemm4 fragment schedule A/B)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash scripts/experiments/r10g.sh && bash scripts/experiments/r10k.sh
