#!/usr/bin/env python3
"""Micro-benchmark of the grouped MoE GEMM (gemm4 MoE mode) on the Mixtral 8x7B
decode shapes: routed gate/up (SwiGLU into per-slot h) and down (weighted atomics into y), at
M tokens with top-2 of 8 experts, random router logits.  Weights cold: the timed loop cycles
through enough copies of the expert stack to defeat the 256 MiB Infinity Cache.  One JSON line per
(phase, M, knob setting); a target for rocprofv3 --pmc passes.

    python tools/moe_bench.py --M 64,256 --knob GEMM4_MOE64=0,1
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mipipe import _native as N  # noqa: E402
from mipipe.ops.kernels import EPI_ATOMIC, EPI_SWIGLU, moe_route, pack_type, packed_dims  # noqa: E402
from mipipe.utils import quants as Q  # noqa: E402

E, K_TOP, D, F = 8, 2, 4096, 14336


def st():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def experts(L, qt, n, k, copies, seed):
    pt = pack_type(qt)
    nbytes = L.mp_packed_bytes(qt, n, k)
    stacks = []
    for c in range(copies):
        W = torch.empty(E * nbytes, dtype=torch.uint8, device="cuda")
        for e in range(E):
            L.mp_init_packed(ctypes.c_void_p(W.data_ptr() + e * nbytes), nbytes, pt, 1.0 / k ** 0.5,
                             seed + 31 * c + e, st())
        stacks.append(W)
    return stacks, pt, nbytes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="256")
    ap.add_argument("--phases", default="gateup,down")
    ap.add_argument("--down-type", default="Q6_K", choices=["Q4_K", "Q6_K"])
    ap.add_argument("--knob", action="append", default=[], metavar="NAME=V[,V..]")
    ap.add_argument("--iters", type=int, default=16)
    ap.add_argument("--copies", type=int, default=3, help="expert stacks cycled (3 x 528 MB defeats the MALL)")
    a = ap.parse_args()
    L = N.lib()
    knobs = [[]]
    for kv in a.knob:
        name, vals = kv.split("=", 1)
        knobs = [kk + [(name, int(v))] for kk in knobs for v in vals.split(",")]
    dqt = Q.Q6_K if a.down_type == "Q6_K" else Q.Q4_K
    gu, gpt, gbytes = experts(L, Q.Q4_K, 2 * F, D, a.copies, 7)
    dn, dpt, dbytes = experts(L, dqt, D, F, a.copies, 9)
    _, kg_pad, g_ntiles, g_nsb = packed_dims(Q.Q4_K, 2 * F, D)
    _, kd_pad, d_ntiles, d_nsb = packed_dims(dqt, D, F)
    for M in [int(x) for x in a.M.split(",")]:
        g = torch.Generator().manual_seed(M)
        logits = torch.randn(M, E, generator=g).cuda()
        counts, lists, weights = moe_route(logits, K_TOP)
        x = torch.randn(M, kg_pad, generator=g).half().cuda()
        h = torch.zeros(M * K_TOP, kd_pad, dtype=torch.float16, device="cuda")
        y = torch.zeros(M, D, device="cuda")

        def run(phase, i):
            if phase == "gateup":
                W = gu[i % len(gu)]
                N.check(L.mp_op_moe_gemm4(gpt, EPI_SWIGLU, ctypes.c_void_p(W.data_ptr()), gbytes, g_ntiles, g_nsb,
                                          ctypes.c_void_p(x.data_ptr()), kg_pad, 0, M, E, K_TOP,
                                          ctypes.c_void_p(counts.data_ptr()), ctypes.c_void_p(lists.data_ptr()),
                                          lists.shape[1], ctypes.c_void_p(weights.data_ptr()), None, 0,
                                          ctypes.c_void_p(h.data_ptr()), kd_pad, F, st()), "moe gate/up")
            else:
                W = dn[i % len(dn)]
                N.check(L.mp_op_moe_gemm4(dpt, EPI_ATOMIC, ctypes.c_void_p(W.data_ptr()), dbytes, d_ntiles, d_nsb,
                                          ctypes.c_void_p(h.data_ptr()), kd_pad, 1, M, E, K_TOP,
                                          ctypes.c_void_p(counts.data_ptr()), ctypes.c_void_p(lists.data_ptr()),
                                          lists.shape[1], ctypes.c_void_p(weights.data_ptr()),
                                          ctypes.c_void_p(y.data_ptr()), D, None, 0, D, st()), "moe down")

        for kn in knobs:
            for name, v in kn:
                N.check(L.mp_set_knob(name.encode(), v), "knob")
            for phase in a.phases.split(","):
                for i in range(2):
                    run(phase, i)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(a.iters):
                    run(phase, i)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.iters
                nb = (gbytes if phase == "gateup" else dbytes) * E
                flops = 2.0 * M * K_TOP * (2 * F * D if phase == "gateup" else D * F)
                print(json.dumps(dict(phase=phase, M=M, knobs=dict(kn) or None, us=round(us, 1),
                                      weight_GBps=round(nb / us / 1e3, 1), TFLOPs=round(flops / us / 1e6, 1))),
                      flush=True)


if __name__ == "__main__":
    main()
