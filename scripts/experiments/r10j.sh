#!/bin/bash
# r10j: chained o -> gate/up -> down (r10g) + 64-row micro-batches on gemm4 (r10i)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash scripts/experiments/r10g.sh && bash scripts/experiments/r10i.sh
