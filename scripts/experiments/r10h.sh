#!/bin/bash
# r10h: r10g (chain) + r10f (MoE weight DMA A/B)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash scripts/experiments/r10g.sh && bash scripts/experiments/r10f.sh
