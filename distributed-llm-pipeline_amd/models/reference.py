"""Pure-PyTorch fp32 reference Llama (the numerics oracle, SURVEY.md §4 tier T2).

Implements exactly the forward of SURVEY.md §3.5 (what llama.cpp's `llm_build_llama` computes for
the reference run, upstream; not in mount): RMSNorm, RoPE "NORM" mode (adjacent pairs) with
optional Llama-3.1 frequency factors, GQA attention with a KV cache, SwiGLU FFN or Mixtral top-k
MoE, final norm + LM head.  Weights are dequantized from the GGUF with the numpy reference
dequantizers, so engine-vs-oracle differences measure kernel numerics only.
"""
from __future__ import annotations

import numpy as np
import torch

from ..utils.gguf import GGUFReader


class RefLlama:
    def __init__(self, tensors: dict, hp: dict, dtype=torch.float32, device="cpu"):
        self.hp = hp
        self.dtype = dtype
        self.device = device
        self.t = {k: torch.as_tensor(np.ascontiguousarray(v)).to(device=device, dtype=dtype)
                  for k, v in tensors.items()}
        d = hp["d_model"]
        self.hd = hp["head_dim"]
        self.n_head, self.n_kv = hp["n_head"], hp["n_head_kv"]
        self.L = hp["n_layer"]
        self.eps = hp["eps"]
        inv = hp["rope_base"] ** (-np.arange(0, self.hd, 2, dtype=np.float64) / self.hd)
        if "rope_freqs.weight" in tensors:
            inv = inv / np.asarray(tensors["rope_freqs.weight"], np.float64)
        self.inv_freq = inv
        if "output.weight" not in self.t:
            self.t["output.weight"] = self.t["token_embd.weight"]
        self.cache_k = [None] * self.L
        self.cache_v = [None] * self.L
        self.kv_round = None   # optional f(t) applied to new K (after RoPE) and V before caching

    @classmethod
    def from_gguf(cls, path: str, dtype=torch.float32, device="cpu"):
        r = GGUFReader(path)
        a = r.kv.get("general.architecture", "llama")
        g = lambda k, dflt=None: r.kv.get(f"{a}.{k}", dflt)
        hp = dict(n_layer=int(g("block_count")), d_model=int(g("embedding_length")),
                  n_head=int(g("attention.head_count")), n_head_kv=int(g("attention.head_count_kv")),
                  d_ff=int(g("feed_forward_length")), rope_base=float(g("rope.freq_base", 10000.0)),
                  eps=float(g("attention.layer_norm_rms_epsilon", 1e-5)),
                  n_expert=int(g("expert_count", 0)), n_expert_used=int(g("expert_used_count", 0)))
        hp["head_dim"] = int(g("rope.dimension_count", hp["d_model"] // hp["n_head"]))
        hp["rope_neox"] = a == "qwen2"   # llama.cpp LLM_ARCH_QWEN2 uses LLAMA_ROPE_TYPE_NEOX
        tensors = {name: r.tensor_f32(name) for name in r.tensors}
        return cls(tensors, hp, dtype, device)

    # ------------------------------------------------------------------ ops
    def rmsnorm(self, x, w):
        x = x * torch.rsqrt((x * x).mean(-1, keepdim=True) + self.eps)
        return x * w

    def rope(self, x, pos):
        # x: [T, H, hd]; Llama: adjacent pairs (2i, 2i+1); NEOX (Qwen2): pairs (i, i + hd/2)
        ang = torch.as_tensor(np.outer(np.asarray(pos, np.float64), self.inv_freq),
                              dtype=torch.float64, device=x.device)
        c, s = torch.cos(ang).to(x.dtype)[:, None, :], torch.sin(ang).to(x.dtype)[:, None, :]
        out = torch.empty_like(x)
        if self.hp.get("rope_neox"):
            h = x.shape[-1] // 2
            x0, x1 = x[..., :h], x[..., h:]
            out[..., :h] = x0 * c - x1 * s
            out[..., h:] = x0 * s + x1 * c
            return out
        x0, x1 = x[..., 0::2], x[..., 1::2]
        out[..., 0::2] = x0 * c - x1 * s
        out[..., 1::2] = x0 * s + x1 * c
        return out

    def reset(self):
        self.cache_k = [None] * self.L
        self.cache_v = [None] * self.L

    @torch.no_grad()
    def forward(self, tokens, start_pos: int, layers=None, x_in=None, want_logits=True):
        """tokens: list[int] (T new tokens at positions start_pos..start_pos+T-1).
        layers: optional (a, b) half-open layer range (pipeline-stage oracle).
        x_in: hidden state input instead of embedding (stage > 0).
        Returns logits [T, vocab] (or hidden state if want_logits is False)."""
        t = self.t
        T = len(tokens) if x_in is None else x_in.shape[0]
        pos = list(range(start_pos, start_pos + T))
        a, b = layers if layers is not None else (0, self.L)
        if x_in is None:
            x = t["token_embd.weight"][torch.as_tensor(tokens, dtype=torch.long, device=self.device)]
        else:
            x = x_in.to(self.dtype)
        hd, H, Hk = self.hd, self.n_head, self.n_kv
        for i in range(a, b):
            p = f"blk.{i}."
            h = self.rmsnorm(x, t[p + "attn_norm.weight"])
            q, k, v = (h @ t[p + "attn_q.weight"].T), (h @ t[p + "attn_k.weight"].T), (h @ t[p + "attn_v.weight"].T)
            if p + "attn_q.bias" in t:
                q, k, v = q + t[p + "attn_q.bias"], k + t[p + "attn_k.bias"], v + t[p + "attn_v.bias"]
            q, k, v = q.view(T, H, hd), k.view(T, Hk, hd), v.view(T, Hk, hd)
            q, k = self.rope(q, pos), self.rope(k, pos)
            if self.kv_round is not None:   # e.g. the fp8 KV cache's rounding
                k, v = self.kv_round(k), self.kv_round(v)
            if self.cache_k[i] is None or start_pos == 0:
                self.cache_k[i], self.cache_v[i] = k, v
            else:
                self.cache_k[i] = torch.cat([self.cache_k[i][:start_pos], k], 0)
                self.cache_v[i] = torch.cat([self.cache_v[i][:start_pos], v], 0)
            K, V = self.cache_k[i], self.cache_v[i]          # [S, Hk, hd]
            S = K.shape[0]
            rep = H // Hk
            Kx = K.repeat_interleave(rep, dim=1)             # [S, H, hd]
            Vx = V.repeat_interleave(rep, dim=1)
            sc = torch.einsum("thd,shd->hts", q, Kx) / np.sqrt(hd)
            qpos = torch.as_tensor(pos, device=self.device)[:, None]
            kpos = torch.arange(S, device=self.device)[None, :]
            sc = sc.masked_fill((kpos > qpos)[None], float("-inf"))
            pr = torch.softmax(sc, dim=-1)
            o = torch.einsum("hts,shd->thd", pr, Vx).reshape(T, H * hd)
            x = x + o @ t[p + "attn_output.weight"].T
            h = self.rmsnorm(x, t[p + "ffn_norm.weight"])
            if self.hp.get("n_expert", 0):
                x = x + self._moe(h, p)
            else:
                g = h @ t[p + "ffn_gate.weight"].T
                u = h @ t[p + "ffn_up.weight"].T
                x = x + (torch.nn.functional.silu(g) * u) @ t[p + "ffn_down.weight"].T
        if not want_logits or b < self.L:
            return x
        h = self.rmsnorm(x, t["output_norm.weight"])
        return h @ t["output.weight"].T

    def _moe(self, h, p):
        t = self.t
        E, k = self.hp["n_expert"], self.hp["n_expert_used"]
        logits = h @ t[p + "ffn_gate_inp.weight"].T          # [T, E]
        probs = torch.softmax(logits, -1)
        w, idx = torch.topk(probs, k, dim=-1)
        w = w / w.sum(-1, keepdim=True)
        out = torch.zeros_like(h)
        G, U, D = t[p + "ffn_gate_exps.weight"], t[p + "ffn_up_exps.weight"], t[p + "ffn_down_exps.weight"]
        for ti in range(h.shape[0]):
            for j in range(k):
                e = int(idx[ti, j])
                g = h[ti] @ G[e].T
                u = h[ti] @ U[e].T
                out[ti] += w[ti, j] * ((torch.nn.functional.silu(g) * u) @ D[e].T)
        return out

    @torch.no_grad()
    def greedy(self, prompt, n_new: int):
        self.reset()
        logits = self.forward(prompt, 0)
        out = []
        nxt = int(torch.argmax(logits[-1]))
        pos = len(prompt)
        for _ in range(n_new):
            out.append(nxt)
            logits = self.forward([nxt], pos)
            pos += 1
            nxt = int(torch.argmax(logits[-1]))
        return out
