#!/usr/bin/env python3
"""Prompt-GEMM design probe: for the 70B / 8B shapes at M rows, time
  (a) the in-kernel-dequant GEMM v2 (launch_gemm2),
  (b) unpack (T16 Q4_K -> f16 [N][K], launch_unpack) + torch f16 matmul (hipBLASLt),
so the choice of a library GEMM behind a per-chunk dequant is measured, not guessed.
Prints one JSON line per shape."""
import argparse, ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mipipe import _native as N
from mipipe.ops.kernels import pack_type, packed_dims, EPI_STORE
from mipipe.utils import quants as Q

SHAPES = {"70b.gateup": (57344, 8192), "70b.down": (8192, 28672), "70b.qkv": (10240, 8192), "70b.o": (8192, 8192),
          "8b.gateup": (28672, 4096), "8b.down": (4096, 14336), "8b.qkv": (6144, 4096)}


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--M", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    L = N.lib()
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    qt = Q.Q4_K
    pt = pack_type(qt)
    for name in a.shapes.split(","):
        n, k = SHAPES[name]
        n_pad, k_pad, ntiles, nsb = packed_dims(qt, n, k)
        nbytes = L.mp_packed_bytes(qt, n, k)
        W = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        L.mp_init_packed(ctypes.c_void_p(W.data_ptr()), nbytes, pt, 1.0 / k ** 0.5, 11, st())
        X = torch.randn(a.M, k_pad, device="cuda").half()
        Y = torch.zeros(a.M, n, device="cuda")
        Wf = torch.empty(ntiles * 16, k_pad, device="cuda", dtype=torch.float16)

        def v2():
            N.check(L.mp_op_gemm2(pt, EPI_STORE, ctypes.c_void_p(W.data_ptr()), ntiles, nsb, ctypes.c_void_p(X.data_ptr()),
                                  k_pad, a.M, ctypes.c_void_p(Y.data_ptr()), n, None, 0, n, st()), "gemm2")

        def unpack():
            N.check(L.mp_op_unpack(pt, ctypes.c_void_p(W.data_ptr()), ntiles, nsb, ctypes.c_void_p(Wf.data_ptr()), k_pad,
                                   st()), "unpack")

        def lib():
            torch.matmul(X, Wf.T, out=Yh)

        Yh = torch.empty(a.M, ntiles * 16, device="cuda", dtype=torch.float16)
        t_v2 = timeit(v2, a.iters)
        t_up = timeit(unpack, a.iters)
        t_mm = timeit(lib, a.iters)
        fl = 2.0 * a.M * n * k
        print(json.dumps(dict(shape=name, M=a.M, gemm2_us=round(t_v2, 1), gemm2_TF=round(fl / t_v2 / 1e6, 1),
                              unpack_us=round(t_up, 1), unpack_GBps=round((nbytes + Wf.numel() * 2) / t_up / 1e3, 1),
                              hipblaslt_us=round(t_mm, 1), hipblaslt_TF=round(fl / t_mm / 1e6, 1),
                              unpack_plus_lib_us=round(t_up + t_mm, 1))), flush=True)
        del W, X, Y, Wf, Yh
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
