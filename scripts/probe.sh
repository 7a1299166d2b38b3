#!/bin/bash
fmt='import sys,json
for l in sys.stdin:
    if not l.startswith("{"): continue
    d=json.loads(l); print(d["shape"],d["type"],"M=%d tpw=%d split=%d %7.1fus %6.0f GB/s"%(d["M"],d["tpw"],d["nsplit"],d["us"],d["GBps"]))'
echo "== probe (loads only)"
timeout -k 10 200 python tools/gemv_bench.py --shapes 70b.gateup --types Q4_K,Q6_K,Q8_0 --M 1 --tpw 1,2,4 --probe 2>&1 | python3 -c "$fmt" || exit 1
echo "== real"
timeout -k 10 200 python tools/gemv_bench.py --shapes 70b.gateup --types Q4_K,Q6_K,Q8_0 --M 1,16 --tpw 1,4 2>&1 | python3 -c "$fmt" || exit 1
