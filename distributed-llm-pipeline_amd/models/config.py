"""Model shapes for the Llama-family configs named in BASELINE.json / SURVEY.md §2.8.

The reference runs `baronllm-llama3.1-v1-q6_k.gguf` (Llama-3.1-8B, `orchestrator/src/main.rs:40`)
and its UI is titled "Stories-15M" (`orchestrator/static/index.html:36`); BASELINE.json adds
TinyLlama-1.1B, Llama-3-70B and Mixtral-8x7B.  Dims are from the public model cards
(SURVEY.md §2.8 table).
"""
from __future__ import annotations

from dataclasses import dataclass, asdict, replace

from ..utils import quants as Q


@dataclass(frozen=True)
class LlamaConfig:
    name: str
    n_layer: int
    d_model: int
    n_head: int
    n_head_kv: int
    d_ff: int
    vocab: int
    rope_base: float = 10000.0
    eps: float = 1e-5
    n_ctx_train: int = 2048
    n_expert: int = 0
    n_expert_used: int = 0
    head_dim: int = 0           # 0 -> d_model // n_head
    tokenizer: str = "llama"    # "gpt2" (byte-level BPE) or "llama" (SPM)
    rope_freq_factors: bool = False   # Llama-3.1 rope_freqs.weight
    arch: str = "llama"         # GGUF general.architecture: "llama" or "qwen2"
    qkv_bias: bool = False      # Qwen2: attn_{q,k,v}.bias
    tied_output: bool = False   # no output.weight (LM head = token_embd)

    @property
    def hd(self) -> int:
        return self.head_dim or self.d_model // self.n_head

    def as_dict(self):
        return asdict(self)

    def scaled(self, **kw) -> "LlamaConfig":
        return replace(self, **kw)


CONFIGS = {
    "stories15m": LlamaConfig("stories15m", 6, 288, 6, 6, 768, 32000, 10000.0, 1e-5, 256),
    "tinyllama": LlamaConfig("tinyllama", 22, 2048, 32, 4, 5632, 32000, 10000.0, 1e-5, 2048),
    "llama3-8b": LlamaConfig("llama3-8b", 32, 4096, 32, 8, 14336, 128256, 500000.0, 1e-5, 8192,
                             tokenizer="gpt2", rope_freq_factors=True),
    "llama3-70b": LlamaConfig("llama3-70b", 80, 8192, 64, 8, 28672, 128256, 500000.0, 1e-5, 8192,
                              tokenizer="gpt2", rope_freq_factors=True),
    "mixtral-8x7b": LlamaConfig("mixtral-8x7b", 32, 4096, 32, 8, 14336, 32000, 1e6, 1e-5, 32768,
                                n_expert=8, n_expert_used=2),
    "qwen2-7b": LlamaConfig("qwen2-7b", 28, 3584, 28, 4, 18944, 152064, 1e6, 1e-6, 32768,
                            tokenizer="gpt2", arch="qwen2", qkv_bias=True),
    # small test shapes (same code paths, fast to generate)
    "tiny-gqa": LlamaConfig("tiny-gqa", 4, 512, 8, 2, 1024, 2048, 10000.0, 1e-5, 1024),
    "tiny-moe": LlamaConfig("tiny-moe", 3, 512, 8, 2, 768, 2048, 10000.0, 1e-5, 1024,
                            n_expert=4, n_expert_used=2),
    "tiny-qwen2": LlamaConfig("tiny-qwen2", 4, 512, 8, 2, 1024, 4096, 1e6, 1e-6, 1024,
                              tokenizer="gpt2", arch="qwen2", qkv_bias=True, tied_output=True),
    "tiny-l3": LlamaConfig("tiny-l3", 4, 1024, 8, 2, 2048, 4096, 500000.0, 1e-5, 1024,
                           tokenizer="gpt2", rope_freq_factors=True),
}


def use_more_bits(i: int, n: int) -> bool:
    """llama.cpp's Q4_K_M layer-promotion rule (upstream; not in mount)."""
    return i < n // 8 or i >= 7 * n // 8 or (i - n // 8) % 3 == 2


def tensor_type(ftype: str, name: str, layer: int, n_layer: int, k_dim: int) -> int:
    """ggml type of a 2-D weight under a named file type (mix)."""
    ftype = ftype.upper()
    plain = {"F32": Q.F32, "F16": Q.F16, "BF16": Q.BF16, "Q8_0": Q.Q8_0, "Q6_K": Q.Q6_K,
             "Q5_K": Q.Q5_K, "Q4_0": Q.Q4_0}
    kq = k_dim % 256 == 0
    if ftype in plain:
        t = plain[ftype]
        if t in (Q.Q6_K, Q.Q5_K) and not kq:
            return Q.Q8_0
        return t
    if ftype in ("Q4_K", "Q4_K_S"):
        if not kq:
            return Q.Q8_0
        return Q.Q6_K if name == "output" else Q.Q4_K
    if ftype == "Q4_K_M":
        if not kq:
            return Q.Q8_0
        if name == "output":
            return Q.Q6_K
        if name in ("attn_v", "ffn_down") and use_more_bits(layer, n_layer):
            return Q.Q6_K
        return Q.Q4_K
    if ftype == "Q5_K_M":
        if not kq:
            return Q.Q8_0
        if name == "output":
            return Q.Q6_K
        if name in ("attn_v", "ffn_down") and use_more_bits(layer, n_layer):
            return Q.Q6_K
        return Q.Q5_K
    raise ValueError(ftype)
