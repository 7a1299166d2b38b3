"""T4 transport tests on one MI355X: the RCCL path of the stage links at world size 1,
torch.distributed's "nccl" (= RCCL) backend in the same process as libmipipe.so, and the 2-byte
stage-boundary wire format (act_dtype) of the piped ring.

The reference's only inter-stage channel is llama.cpp's ggml-rpc over TCP
(orchestrator/src/main.rs:47-48, `--rpc 127.0.0.1:50052,127.0.0.1:50053`); ours is RCCL
ncclSend/ncclRecv over xGMI.  Multi-rank RCCL needs one GPU per rank, so on the 1-GPU box the
RcclLink is exercised as a self loop (1-rank communicator, grouped send + recv) and the multi-rank
wiring is covered by the CPU multi-process tests (gloo / TCP) of test_parallel.py."""
import ctypes
import json
import socket

import numpy as np
import pytest
import torch

from conftest import make_model

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _selftest(native, sizes, iters=3):
    from mipipe import _native as N
    arr = (ctypes.c_int64 * len(sizes))(*sizes)
    return N.jcall(native.mp_rccl_selftest, 0, ctypes.cast(arr, ctypes.c_void_p), len(sizes), iters,
                   what="rccl selftest")


def test_rccl_link_self_loop(cuda, native):
    """RcclLink (the engine's stage link class) over a 1-rank communicator: every message size the
    pipeline uses (token ids, one bf16 70B row, a 64-row micro-batch, a 512-row prefill chunk)
    arrives intact and is counted."""
    sizes = [4, 64 * 4, 8192 * 2, 64 * 8192 * 2, 512 * 8192 * 2 + 6]
    rep = _selftest(native, sizes, iters=3)
    assert rep["ok"], rep
    assert rep["bytes_sent"] == 3 * sum(sizes) and rep["msgs_sent"] == 3 * len(sizes)
    assert rep["rccl_version"].count(".") == 2
    print("RCCL_SELFTEST " + json.dumps(rep))


def test_rccl_side_stream_loop(cuda, native):
    """The CU-sharing proxy (mp_rccl_loop_start / wait, tools/gemv_bench.py --rccl-bytes): RCCL self
    send/recv of a 256 x 8192 bf16 activation queued on a side stream runs while the caller's stream
    computes, and reports its wall time."""
    import torch
    assert native.mp_rccl_loop_start(0, 256 * 8192 * 2, 20) == 0, native.mp_last_error()
    a = torch.randn(4096, 4096, device="cuda")
    for _ in range(4):
        a = a @ a.T / 64.0
    torch.cuda.synchronize()
    ms = native.mp_rccl_loop_wait()
    assert ms > 0, native.mp_last_error()


def test_torch_nccl_world1_with_native_lib(cuda, native):
    """torch.distributed backend "nccl" (RCCL on ROCm) at world size 1, in the process that has
    libmipipe.so (sharing torch's HIP runtime and librccl): collectives work, then our own RCCL
    communicator works beside it, then an engine runs."""
    import torch.distributed as dist
    from mipipe.engine import Engine, rccl_unique_id_hex
    assert not dist.is_initialized()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        x = torch.arange(1024, dtype=torch.float32, device="cuda")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        assert torch.equal(x.cpu(), torch.arange(1024, dtype=torch.float32))
        ids = [None]
        dist.all_gather_object(ids, rccl_unique_id_hex())   # the id exchange of init_from_torchrun
        assert len(bytes.fromhex(ids[0])) == 128
        rep = _selftest(native, [4096, 1 << 20], iters=2)
        assert rep["ok"], rep
        syn = dict(n_layer=2, d_model=512, n_head=8, n_head_kv=2, d_ff=1024, vocab=2048, rope_base=10000.0)
        with Engine(synthetic=syn, ftype="Q4_K", max_ctx=128, mb_size=2) as eng:
            out, _ = eng.generate([[1, 2, 3], [4, 5]], 4)
        assert all(len(o) == 4 for o in out)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_rccl_two_ranks_one_gpu_probe_or_pipeline(cuda, native, model_dir):
    """If RCCL accepts two ranks on the one GPU, run the real RcclLink pipeline (PP=2, local mode)
    against PP=1; RCCL normally refuses a duplicate GPU, which is reported, not hidden."""
    from mipipe import _native as N
    from mipipe.engine import Engine
    devs = (ctypes.c_int * 2)(0, 0)
    probe = N.jcall(native.mp_rccl_probe_devices, ctypes.cast(devs, ctypes.c_void_p), 2, what="probe")
    if not probe["ok"]:
        pytest.skip("RCCL refuses two ranks on one GPU: " + probe["error"])
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    prompts = [[3, 4, 5, 6], [7, 8], [9, 10, 11], [12]]
    with Engine(gguf=path, max_ctx=64, n_mb=2, mb_size=2) as eng:
        ref_out, _ = eng.generate(prompts, 7)
    with Engine(gguf=path, max_ctx=64, n_mb=2, mb_size=2, stages=2, devices=[0, 0], link="rccl",
                act_dtype="f32", split="even") as eng:
        out, _ = eng.generate(prompts, 7)
    assert out == ref_out


@pytest.mark.parametrize("wire", ["bf16", "f16"])
def test_two_byte_stage_boundary(cuda, native, model_dir, wire):
    """act_dtype bf16 / f16: stage boundaries carry d_model x 2 bytes per token and the
    pipeline's logits stay close to the f32-boundary pipeline (rounding the residual once per
    boundary).  PP=2 emulated on one GPU with LocalLinks."""
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    rng = np.random.default_rng(4)
    prompts = [[int(t) for t in rng.integers(3, cfg.vocab, n)] for n in (9, 14)]
    kw = dict(gguf=path, max_ctx=128, n_mb=1, mb_size=2, prefill_chunk=16, stages=2, devices=[0, 0],
              link="local", split="even")
    logits = {}
    for ad in ("f32", wire):
        with Engine(act_dtype=ad, **kw) as eng:
            eng.start(prompts)
            logits[ad] = eng.logits(2).copy()   # prompt logits: no sampled token feeds back yet
            eng.decode(3)
            h = eng.health()
            st0 = [s for s in h["stages"] if s["stage"] == 0][0]
            # stage 0 -> 1: prompt rows (chunks) + 3 decode rounds x 2 rows, at 2 or 4 bytes each
            rows = sum(len(p) for p in prompts) + 3 * 2
            assert st0["bytes_sent"] == rows * cfg.d_model * (4 if ad == "f32" else 2), (ad, st0)
    a, b = logits["f32"].astype(np.float64), logits[wire].astype(np.float64)
    err = ((a - b) ** 2).sum() / (a ** 2).sum()
    assert err < (1e-4 if wire == "bf16" else 1e-6), err
