"""hipBLASLt (torch f16 / bf16 matmul on plain 16-bit weights, no dequant) at the Llama-3 projection
shapes: the library yardstick for the dequant GEMMs (gemm2 / gemm3).  Weights are cycled through
enough copies to defeat the 256 MiB MALL, like tools/gemv_bench.py.

    python tools/torch_mm_probe.py --M 256,512 [--dtype bf16]
"""
import argparse

import torch

SHAPES = {"70b.qkv": (10240, 8192), "70b.o": (8192, 8192), "70b.gateup": (57344, 8192), "70b.down": (8192, 28672),
          "8b.gateup": (28672, 4096), "8b.down": (4096, 14336)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="256")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--dtype", default="f16", choices=["f16", "bf16"])
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dt = torch.float16 if a.dtype == "f16" else torch.bfloat16
    torch.manual_seed(0)
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        copies = max(2, min(8, (1536 << 20) // (N * K * 2) + 1))
        ws = [torch.randn(N, K, device="cuda", dtype=dt) for _ in range(copies)]
        for M in [int(m) for m in a.M.split(",")]:
            x = torch.randn(M, K, device="cuda", dtype=dt)
            for w in ws[:2]:
                y = x @ w.T
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(a.iters):
                y = x @ ws[i % copies].T
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.iters
            print(f'{{"shape": "{name}", "op": "torch.matmul {a.dtype}", "M": {M}, "us": {us:.2f}, '
                  f'"TFLOPs": {2 * M * N * K / us / 1e6:.1f}}}', flush=True)
            del y
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
