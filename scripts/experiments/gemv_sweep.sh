#!/bin/bash
mkdir -p gpurun_out
fmt='import sys,json
for l in sys.stdin:
    if not l.startswith("{"): continue
    d=json.loads(l); print(d["shape"],d["type"],"M=%d tpw=%d split=%d %7.1fus %6.0f GB/s"%(d["M"],d["tpw"],d["nsplit"],d["us"],d["GBps"]))'
timeout -k 10 200 python tools/gemv_bench.py --shapes 70b.gateup,70b.head --types Q4_K --M 1,16 --tpw 1,2,4 2>&1 | python3 -c "$fmt" || exit 1
timeout -k 10 300 python tools/gemv_bench.py --shapes 70b.qkv,70b.o,70b.down --types Q4_K --M 1,16 --tpw 1,2,4 --splits 1,2,4,8 2>&1 | python3 -c "$fmt" || exit 1
