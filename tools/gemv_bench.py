#!/usr/bin/env python3
"""Micro-benchmark of the dequant-GEMV kernel on the Llama-3-70B / 8B decode shapes.

Weights are COLD like in a real decode step: the timed loop cycles through enough copies of the
matrix (>= 1.5 GB) that the 256 MiB Infinity Cache cannot serve them (a single re-streamed matrix
that fits the MALL reads up to 40 % faster than HBM allows).  Reports weight GB/s per
(shape, type, M, tiles-per-wave, split)."""
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
    "8b.qkv": (6144, 4096, EPI_ATOMIC), "8b.o": (4096, 4096, EPI_ATOMIC),
    "8b.gateup": (28672, 4096, EPI_SWIGLU), "8b.down": (4096, 14336, EPI_ATOMIC),
}
TYPES = {"Q4_K": Q.Q4_K, "Q6_K": Q.Q6_K, "Q8_0": Q.Q8_0, "Q5_K": Q.Q5_K, "F16": Q.F16, "BF16": Q.BF16}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="70b.qkv,70b.o,70b.gateup,70b.down,70b.head")
    ap.add_argument("--types", default="Q4_K")
    ap.add_argument("--M", default="1,16")
    ap.add_argument("--tpw", default="0", help="tiles per wave at M > 32: 0 auto, 1, 2")
    ap.add_argument("--splits", default="auto")
    ap.add_argument("--iters", type=int, default=24)
    ap.add_argument("--target", type=int, default=2048)
    ap.add_argument("--epi", type=int, default=-1, help="override the epilogue (0 store, 1 atomic): timing probes")
    ap.add_argument("--copies", type=int, default=0, help="weight copies cycled (default: enough to defeat the 256 MiB MALL; 1 = hot)")
    ap.add_argument("--gemm", type=int, default=0,
                    help="time the prompt GEMM instead (1: 64x64 tiles, 2: 128x256 per-wave dequant, 3: LDS-shared dequant, "
                         "4: gemm3's stream on the 32x32x16 MFMA, 8: the int8-activation prototype on per-row int8 "
                         "weights, gemm3 P_I8)")
    ap.add_argument("--sk", action="store_true",
                    help="ATOMIC shapes with --gemm 2 / 4: the engine's split-K (per-split partial stores + the "
                         "fixed-order reduction into Y) instead of atomics")
    ap.add_argument("--g3", default="0,0,0", help="v3 GEMM tuning BM,BN,nsplit (0 = auto); ';'-separated list sweeps")
    ap.add_argument("--knob", action="append", default=[], metavar="NAME=V[,V..]",
                    help="tuning knob (csrc/runtime/tuning.h) swept per shape, e.g. GEMM3_PROBE=0,1,2")
    ap.add_argument("--rccl-bytes", type=int, default=0,
                    help="CU-sharing proxy: run each timed loop twice, the second time with a 1-rank RCCL self "
                         "send/recv loop of this many bytes on a side stream (mp_rccl_loop_start)")
    a = ap.parse_args()
    L = N.lib()
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for sname in a.shapes.split(","):
        n, k, epi = SHAPES[sname]
        if a.epi >= 0:
            epi = a.epi
        for tname in a.types.split(","):
            qt = TYPES[tname]
            if sname.endswith("head") and tname == "Q4_K":
                qt, tname = Q.Q6_K, "Q6_K"
            pt = pack_type(qt)
            n_pad, k_pad, ntiles, nsb = packed_dims(qt, n, k)
            nbytes = L.mp_packed_bytes(qt, n, k)
            if a.gemm == 8:   # int8 weights: 1 byte per element, per-row scales
                tname, nbytes = "I8", ntiles * nsb * 4096
            copies = a.copies or max(2, min(24, (1536 << 20) // nbytes + 1))
            Ws = []
            for c in range(copies):
                if a.gemm == 8:
                    Ws.append(torch.randint(-127, 128, (nbytes,), dtype=torch.int8, device="cuda"))
                    continue
                W = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
                L.mp_init_packed(ctypes.c_void_p(W.data_ptr()), nbytes, pt, 1.0 / k ** 0.5, 7 + c, st())
                Ws.append(W)
            ws = torch.full((ntiles * 16,), 1e-3, device="cuda")
            for M in [int(x) for x in a.M.split(",")]:
                X = torch.randn(M, k_pad, device="cuda").half()
                Xq = torch.randint(-127, 128, (M, k_pad), dtype=torch.int8, device="cuda")
                xs = torch.full((M,), 1e-2, device="cuda")
                Y = torch.zeros(M, n, device="cuda")
                H = torch.zeros(M, n // 2, device="cuda", dtype=torch.float16)
                SK = torch.empty(16 * M * ntiles * 16 if a.sk else 1, device="cuda")
                knobs = [[]]
                for kv in a.knob:
                    name, vals = kv.split("=", 1)
                    knobs = [k + [(name, int(v))] for k in knobs for v in vals.split(",")]
                for tpw, g3, kn in [(int(t), g, k) for t in a.tpw.split(",") for g in a.g3.split(";") for k in knobs]:
                    L.mp_set_gemv_tpw(tpw)
                    bm, bn, g3s = [int(v) for v in g3.split(",")]
                    # (0 arguments reset GEMM3_BM / BN / SPLIT to their defaults: --knob values go after)
                    L.mp_set_gemm3_tuning(bm, bn, g3s, 0)
                    for name, v in kn:
                        N.check(L.mp_set_knob(name.encode(), v), "set_knob")
                    waves = (ntiles + max(tpw, 1) - 1) // max(tpw, 1)
                    if a.gemm or epi == EPI_SWIGLU or (epi != EPI_ATOMIC and a.splits == "auto"):
                        splits = [1]
                    elif a.splits == "auto":
                        splits = [max(1, min((a.target + waves - 1) // waves, max(1, nsb // 4)))]
                    else:
                        splits = [int(s) for s in a.splits.split(",")]
                    for nsplit in splits:
                        def run(W):
                            if a.gemm == 8:
                                N.check(L.mp_op_gemm3_i8(epi, ctypes.c_void_p(W.data_ptr()), ntiles, nsb,
                                                         ctypes.c_void_p(Xq.data_ptr()), k_pad, M, ctypes.c_void_p(Y.data_ptr()),
                                                         n, ctypes.c_void_p(H.data_ptr()), n // 2,
                                                         n if epi != EPI_SWIGLU else n // 2, ctypes.c_void_p(xs.data_ptr()),
                                                         ctypes.c_void_p(ws.data_ptr()), 1, st()), "gemm3_i8")
                                return
                            if a.sk and a.gemm in (2, 4) and epi == EPI_ATOMIC:
                                fn = L.mp_op_gemm4_splitk if a.gemm == 4 else L.mp_op_gemm2_splitk
                                N.check(fn(pt, ctypes.c_void_p(W.data_ptr()), ntiles, nsb, ctypes.c_void_p(X.data_ptr()),
                                           k_pad, M, ctypes.c_void_p(Y.data_ptr()), n, n,
                                           ctypes.c_void_p(SK.data_ptr()), SK.numel(), st()), "gemm splitk")
                                return
                            if a.gemm == 4:
                                N.check(L.mp_op_gemm4(pt, epi, ctypes.c_void_p(W.data_ptr()), ntiles, nsb,
                                                      ctypes.c_void_p(X.data_ptr()), k_pad, M, ctypes.c_void_p(Y.data_ptr()),
                                                      n, ctypes.c_void_p(H.data_ptr()), n // 2,
                                                      n if epi != EPI_SWIGLU else n // 2, 1, st()), "gemm4")
                                return
                            if a.gemm == 3:
                                N.check(L.mp_op_gemm3(pt, epi, ctypes.c_void_p(W.data_ptr()), ntiles, nsb,
                                                      ctypes.c_void_p(X.data_ptr()), k_pad, M, ctypes.c_void_p(Y.data_ptr()),
                                                      n, ctypes.c_void_p(H.data_ptr()), n // 2,
                                                      n if epi != EPI_SWIGLU else n // 2, 1, st()), "gemm3")
                                return
                            if a.gemm:
                                fn = L.mp_op_gemm2 if a.gemm == 2 else L.mp_op_gemm
                                N.check(fn(pt, epi, ctypes.c_void_p(W.data_ptr()), ntiles, nsb,
                                           ctypes.c_void_p(X.data_ptr()), k_pad, M, ctypes.c_void_p(Y.data_ptr()),
                                           n, ctypes.c_void_p(H.data_ptr()), n // 2,
                                           n if epi != EPI_SWIGLU else n // 2, st()), "gemm")
                                return
                            N.check(L.mp_op_gemv(pt, epi, ctypes.c_void_p(W.data_ptr()), ntiles, nsb,
                                                 ctypes.c_void_p(X.data_ptr()), k_pad, M, ctypes.c_void_p(Y.data_ptr()),
                                                 n, ctypes.c_void_p(H.data_ptr()), n // 2,
                                                 n if epi != EPI_SWIGLU else n // 2, nsplit, st()), "gemv")
                        for W in Ws[:2]:
                            run(W)
                        torch.cuda.synchronize()
                        for with_rccl in ([False, True] if a.rccl_bytes else [False]):
                            rccl_ms = None
                            if with_rccl:   # side-stream RCCL kernels sharing the CUs for the whole timed loop
                                N.check(L.mp_rccl_loop_start(torch.cuda.current_device(), a.rccl_bytes, 400), "rccl loop")
                            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                            e0.record()
                            for i in range(a.iters):
                                run(Ws[i % copies])
                            e1.record()
                            torch.cuda.synchronize()
                            if with_rccl:
                                rccl_ms = round(L.mp_rccl_loop_wait(), 3)
                            us = e0.elapsed_time(e1) * 1e3 / a.iters
                            print(json.dumps(dict(shape=sname, type=tname, M=M, tpw=tpw, nsplit=nsplit, us=round(us, 2),
                                                  GBps=round(nbytes / us / 1e3, 1),
                                                  TFLOPs=round(2.0 * M * n * k / us / 1e6, 1), gemm=a.gemm,
                                                  g3=g3 if a.gemm in (3, 4, 8) else None, sk=a.sk or None, knobs=dict(kn) or None,
                                                  rccl_bytes=a.rccl_bytes if with_rccl else None,
                                                  rccl_loop_ms=rccl_ms)), flush=True)
                if a.gemm == 8:   # the per-row activation quantization the int8 GEMM needs first
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for i in range(a.iters):
                        N.check(L.mp_op_quant_i8(ctypes.c_void_p(X.data_ptr()), k_pad, M, k_pad,
                                                 ctypes.c_void_p(Xq.data_ptr()), k_pad, ctypes.c_void_p(xs.data_ptr()), st()), "q")
                    e1.record()
                    torch.cuda.synchronize()
                    print(json.dumps(dict(shape=sname, op="quant_rows_i8", M=M, us=round(e0.elapsed_time(e1) * 1e3 / a.iters, 2))),
                          flush=True)
            del Ws
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
