#!/bin/bash
# gemm3<P_I8> tile sweep at the 70B / 8B shapes, M = 256 (cold weights)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python tools/gemv_bench.py --gemm 8 --M 256 --shapes 70b.gateup,70b.qkv,70b.o,70b.down,8b.gateup,8b.down \
  --g3 "0,0,0;128,256,0;128,128,0;256,128,0;256,256,0" > $O/i8_tiles.log 2>&1 || { tail -5 $O/i8_tiles.log; exit 1; }
grep -v quant_rows $O/i8_tiles.log | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], d.get('g3'), d['us'], d.get('TFLOPs'))"
