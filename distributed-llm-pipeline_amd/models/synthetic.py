"""Synthetic random-init GGUF generator for the Llama-family configs.

There is no network for checkpoints, so every model the engine runs in tests and benches is
random-init with the *architecture* of the named model.  Small models
quantize float weights (realistic block statistics); large ones write random quant blocks
directly (`quants.random_blocks`) so an 8B file is produced in seconds.
"""
from __future__ import annotations

import numpy as np

from ..utils import quants as Q
from ..utils.gguf import GGUFWriter, U32, F32T, STRING, I32
from .config import LlamaConfig, tensor_type
from . import tokenizer_data


def llama_tensor_specs(cfg: LlamaConfig, ftype: str):
    """Yield (name, ggml_shape, qtype, kind) for every tensor of the model."""
    d, hd = cfg.d_model, cfg.hd
    L = cfg.n_layer
    yield ("token_embd.weight", (d, cfg.vocab), tensor_type(ftype, "token_embd", 0, L, d), "embd")
    yield ("output_norm.weight", (d,), Q.F32, "norm")
    if not cfg.tied_output:
        yield ("output.weight", (d, cfg.vocab), tensor_type(ftype, "output", 0, L, d), "w")
    if cfg.rope_freq_factors:
        yield ("rope_freqs.weight", (hd // 2,), Q.F32, "rope")
    for i in range(L):
        p = f"blk.{i}."
        yield (p + "attn_norm.weight", (d,), Q.F32, "norm")
        yield (p + "attn_q.weight", (d, cfg.n_head * hd), tensor_type(ftype, "attn_q", i, L, d), "w")
        yield (p + "attn_k.weight", (d, cfg.n_head_kv * hd), tensor_type(ftype, "attn_k", i, L, d), "w")
        yield (p + "attn_v.weight", (d, cfg.n_head_kv * hd), tensor_type(ftype, "attn_v", i, L, d), "w")
        if cfg.qkv_bias:
            yield (p + "attn_q.bias", (cfg.n_head * hd,), Q.F32, "bias")
            yield (p + "attn_k.bias", (cfg.n_head_kv * hd,), Q.F32, "bias")
            yield (p + "attn_v.bias", (cfg.n_head_kv * hd,), Q.F32, "bias")
        yield (p + "attn_output.weight", (cfg.n_head * hd, d),
               tensor_type(ftype, "attn_output", i, L, cfg.n_head * hd), "wo")
        yield (p + "ffn_norm.weight", (d,), Q.F32, "norm")
        if cfg.n_expert:
            yield (p + "ffn_gate_inp.weight", (d, cfg.n_expert), Q.F32, "router")
            yield (p + "ffn_gate_exps.weight", (d, cfg.d_ff, cfg.n_expert),
                   tensor_type(ftype, "ffn_gate", i, L, d), "w")
            yield (p + "ffn_up_exps.weight", (d, cfg.d_ff, cfg.n_expert),
                   tensor_type(ftype, "ffn_up", i, L, d), "w")
            yield (p + "ffn_down_exps.weight", (cfg.d_ff, d, cfg.n_expert),
                   tensor_type(ftype, "ffn_down", i, L, cfg.d_ff), "wo")
        else:
            yield (p + "ffn_gate.weight", (d, cfg.d_ff), tensor_type(ftype, "ffn_gate", i, L, d), "w")
            yield (p + "ffn_up.weight", (d, cfg.d_ff), tensor_type(ftype, "ffn_up", i, L, d), "w")
            yield (p + "ffn_down.weight", (cfg.d_ff, d), tensor_type(ftype, "ffn_down", i, L, cfg.d_ff), "wo")


def _float_init(rng, name, shape, kind, cfg: LlamaConfig, wscale: float):
    n = int(np.prod(shape))
    if kind == "norm":
        return (1.0 + 0.1 * rng.standard_normal(n)).astype(np.float32)
    if kind == "rope":
        # Llama-3.1 style frequency factors: 1 for high freqs, up to 8 for low freqs
        i = np.arange(n)
        return (1.0 + 7.0 * (i / max(n - 1, 1)) ** 2).astype(np.float32)
    if kind == "bias":
        return (rng.standard_normal(n) * 0.5).astype(np.float32)
    if kind == "router":
        return (rng.standard_normal(n) * 0.5).astype(np.float32)
    if kind == "embd":
        return (rng.standard_normal(n) * 1.0).astype(np.float32)
    fan_in = shape[0]
    s = wscale / np.sqrt(fan_in)
    return (rng.standard_normal(n) * s).astype(np.float32)


def write_synthetic_gguf(path: str, cfg: LlamaConfig, ftype: str = "Q4_K_M", seed: int = 0,
                         fast_random_blocks: bool | None = None, wscale: float = 1.0,
                         with_tokenizer: bool = True) -> str:
    """Write a random-init GGUF for `cfg` with file type mix `ftype`."""
    rng = np.random.default_rng(seed)
    if fast_random_blocks is None:
        fast_random_blocks = cfg.d_model >= 2048
    w = GGUFWriter(path)
    arch = cfg.arch
    w.add("general.architecture", arch)
    w.add("general.name", f"synthetic-{cfg.name}-{ftype}")
    w.add("general.file_type", 15 if ftype.upper() == "Q4_K_M" else 0, U32)
    w.add(f"{arch}.block_count", cfg.n_layer, U32)
    w.add(f"{arch}.context_length", cfg.n_ctx_train, U32)
    w.add(f"{arch}.embedding_length", cfg.d_model, U32)
    w.add(f"{arch}.feed_forward_length", cfg.d_ff, U32)
    w.add(f"{arch}.attention.head_count", cfg.n_head, U32)
    w.add(f"{arch}.attention.head_count_kv", cfg.n_head_kv, U32)
    w.add(f"{arch}.rope.freq_base", float(cfg.rope_base), F32T)
    w.add(f"{arch}.rope.dimension_count", cfg.hd, U32)
    w.add(f"{arch}.attention.layer_norm_rms_epsilon", float(cfg.eps), F32T)
    w.add(f"{arch}.vocab_size", cfg.vocab, U32)
    if cfg.n_expert:
        w.add(f"{arch}.expert_count", cfg.n_expert, U32)
        w.add(f"{arch}.expert_used_count", cfg.n_expert_used, U32)
    if with_tokenizer:
        tokenizer_data.add_tokenizer_kv(w, cfg)

    for name, shape, qt, kind in llama_tensor_specs(cfg, ftype):
        n = int(np.prod(shape))
        if fast_random_blocks and qt not in (Q.F32,) and kind in ("w", "wo", "embd"):
            sub = np.random.default_rng(rng.integers(1 << 62))
            scale = 1.0 if kind == "embd" else wscale / np.sqrt(shape[0])
            rows = n // shape[0]

            def gen(sub=sub, qt=qt, rows=rows, k=shape[0], scale=scale):
                return Q.random_blocks(sub, qt, rows, k, scale)
            w.add_tensor(name, gen, qt, shape)
        else:
            x = _float_init(rng, name, shape, kind, cfg, wscale)
            w.add_tensor(name, Q.quantize(x, qt), qt, shape)
    w.write()
    return path
