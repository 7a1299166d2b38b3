#!/usr/bin/env bash
# Weak-scaling curve (N = 1, 2, 4, 8) of bench.py as one JSON line; see scripts/scale.py.
#   bash scripts/scale.sh [--launcher inproc|torchrun] [--gpus 1,2,4,8] [--same-device] [-- bench args]
set -o pipefail
cd "$(dirname "$0")/.." && exec python3 scripts/scale.py "$@"
