import torch, time
torch.manual_seed(0)
for (M, N, K) in [(512, 57344, 8192), (512, 8192, 28672), (512, 10240, 8192), (512, 28672, 4096), (2048, 57344, 8192)]:
    x = torch.randn(M, K, device="cuda", dtype=torch.float16)
    w = torch.randn(N, K, device="cuda", dtype=torch.float16)
    for _ in range(3): y = x @ w.T
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): y = x @ w.T
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 100
    print(f"torch f16 matmul M={M} N={N} K={K}: {us:.1f} us  {2*M*N*K/us/1e6:.0f} TFLOP/s", flush=True)
    del x, w, y
