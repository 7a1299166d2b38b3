#!/usr/bin/env python3
"""Micro-benchmark of the dequant-GEMV kernel on the Llama-3-70B / 8B decode shapes.
Reports achieved weight-stream bandwidth (GB/s) per (shape, type, M, waves-per-block)."""
import argparse, ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mipipe import _native as N
from mipipe.ops.kernels import pack_type, packed_dims, EPI_STORE, EPI_ATOMIC, EPI_SWIGLU
from mipipe.utils import quants as Q

SHAPES = {  # name: (N, K, epi)
    "70b.qkv": (10240, 8192, EPI_ATOMIC), "70b.o": (8192, 8192, EPI_ATOMIC),
    "70b.gateup": (57344, 8192, EPI_SWIGLU), "70b.down": (8192, 28672, EPI_ATOMIC),
    "70b.head": (128256, 8192, EPI_STORE),
    "8b.qkv": (6144, 4096, EPI_ATOMIC), "8b.gateup": (28672, 4096, EPI_SWIGLU), "8b.down": (4096, 14336, EPI_ATOMIC),
}
TYPES = {"Q4_K": Q.Q4_K, "Q6_K": Q.Q6_K, "Q8_0": Q.Q8_0, "Q5_K": Q.Q5_K, "F16": Q.F16}

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="70b.qkv,70b.o,70b.gateup,70b.down,70b.head")
    ap.add_argument("--types", default="Q4_K")
    ap.add_argument("--M", default="1,16")
    ap.add_argument("--wpb", default="1")
    ap.add_argument("--tpw", default="1,2,4")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--target", type=int, default=2048)
    a = ap.parse_args()
    L = N.lib()
    L.mp_set_gemv_wpb.argtypes = [ctypes.c_int]
    res = []
    for sname in a.shapes.split(","):
        n, k, epi = SHAPES[sname]
        for tname in a.types.split(","):
            qt = TYPES[tname]
            if sname.endswith("head") and tname == "Q4_K":
                qt, tname = Q.Q6_K, "Q6_K"
            pt = pack_type(qt)
            n_pad, k_pad, ntiles, nsb = packed_dims(qt, n, k)
            nbytes = L.mp_packed_bytes(qt, n, k)
            W = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
            L.mp_init_packed(ctypes.c_void_p(W.data_ptr()), nbytes, pt, 1.0 / k ** 0.5, 7,
                             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            for M in [int(x) for x in a.M.split(",")]:
                X = torch.randn(M, k_pad, device="cuda").half()
                Y = torch.zeros(M, n, device="cuda")
                H = torch.zeros(M, n // 2, device="cuda", dtype=torch.float16)
                nsplit = 1
                for wpb, tpw in [(int(w), int(t)) for w in a.wpb.split(",") for t in a.tpw.split(",")]:
                    L.mp_set_gemv_tpw(tpw)
                    if epi == EPI_ATOMIC:
                        waves = (ntiles + tpw - 1) // tpw
                        nsplit = max(1, min((a.target + waves - 1) // waves, max(1, nsb // 4)))
                    L.mp_set_gemv_wpb(wpb)
                    def run():
                        N.check(L.mp_op_gemv(pt, epi, ctypes.c_void_p(W.data_ptr()), ntiles, nsb,
                                             ctypes.c_void_p(X.data_ptr()), k_pad, M, ctypes.c_void_p(Y.data_ptr()), n,
                                             ctypes.c_void_p(H.data_ptr()), n // 2, n if epi != EPI_SWIGLU else n // 2,
                                             nsplit, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "gemv")
                    for _ in range(3): run()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters): run()
                    e1.record(); torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) * 1e3 / a.iters
                    r = dict(shape=sname, type=tname, M=M, wpb=wpb, tpw=tpw, nsplit=nsplit, us=round(us, 2),
                             GBps=round(nbytes / us / 1e3, 1))
                    res.append(r)
                    print(json.dumps(r), flush=True)
    return res

if __name__ == "__main__":
    main()
