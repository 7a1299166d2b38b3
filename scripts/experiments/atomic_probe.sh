#!/bin/bash
# cost of the split-K atomic epilogue at M = 64: same GEMVs with plain stores (wrong sums, timing only)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for e in 1 0; do
  echo "== epi=$e"
  timeout -k 10 200 python3 tools/gemv_bench.py --shapes 70b.qkv,70b.o,70b.down --M 16,64 --tpw 1 --splits 1,2,4,8 --epi $e > $O/ap_$e.log 2>&1 || { tail -5 $O/ap_$e.log; exit 1; }
  python3 -c "
import json
for l in open('$O/ap_$e.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], d['M'], d['nsplit'], d['us'])" | paste - - - -
done
for nw in 4; do
  echo "== atomic NW=$nw"
  MIPIPE_GEMV_NW=$nw timeout -k 10 200 python3 tools/gemv_bench.py --shapes 70b.qkv,70b.o,70b.down --M 64 --tpw 1 --splits 1,2,4,8 > $O/ap_nw.log 2>&1 || { tail -5 $O/ap_nw.log; exit 1; }
  python3 -c "
import json
for l in open('$O/ap_nw.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], d['M'], d['nsplit'], d['us'])" | paste - - - -
done
