"""Python front-end of the native pipeline engine (csrc/runtime/engine.cpp).

    eng = Engine(gguf="model.gguf", stages=2, n_mb=2, mb_size=4, max_ctx=2048)
    out, stats = eng.generate([[1, 15, 27], [1, 99]], n_predict=32)

Config keys mirror the C++ Engine (see engine.h): gguf | synthetic+ftype, mode ("local" or "mp"),
stages, devices, link ("local" | "rccl" | "tcp"), backend ("hip" | "cpu"), gpu_layers (llama-cli -ngl N:
0 < N < n_layer puts the first n_layer - N layers on a CPU stage in front of the GPU stages), n_mb, mb_size, max_ctx,
prefill_chunk, split ("even" | "mem" | "cost"), graphs, fused_attn, prefill_gemm, attn_split_len,
temp/top_k/top_p/min_p/seed (sampling; llama.cpp chain order), repeat_penalty/repeat_last_n/
frequency_penalty/presence_penalty (penalties over the last n tokens, prompt included), world/rank/hosts/next_host/base_port/rccl_ids (mp mode),
threads (CPU backend), trace, watchdog_s, link_timeout_s, fault (fault injection), verbose, log_file,
kv_dtype ("f16" | "fp8"), kv_pool_tokens (paged KV pool), prefill_gemm_v (0 auto | 1 | 2 | 3 | 4), prefill_flash,
deterministic, fused_norm, small_gemv, act_dtype (stage-boundary wire: "auto" | "f32" | "bf16" | "f16"),
device_speed ("probe" or a list; Halda-style partition weights).
"""
from __future__ import annotations

import ctypes
import json

import numpy as np

from . import _native as N


class Engine:
    def __init__(self, **cfg):
        self.cfg = dict(cfg)
        L = N.lib()
        h = L.mp_engine_create(N.cstr(json.dumps(self.cfg)))
        if not h:
            N.check(None, "engine create")
        self._h = ctypes.c_void_p(h)
        self.info = N.jcall(L.mp_engine_info, self._h, what="engine info")
        self.n_seq_cap = self.info["n_mb"] * self.info["mb_size"]

    def close(self):
        if getattr(self, "_h", None):
            N.lib().mp_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @staticmethod
    def _flat(prompts):
        lens = np.asarray([len(p) for p in prompts], np.int32)
        flat = np.asarray([t for p in prompts for t in p], np.int32)
        return flat, lens

    def generate(self, prompts, n_predict: int):
        flat, lens = self._flat(prompts)
        out = np.full((len(prompts), n_predict), -1, np.int32)
        stats = N.jcall(N.lib().mp_engine_generate, self._h, flat.ctypes.data, lens.ctypes.data, len(prompts),
                        n_predict, out.ctypes.data, what="generate")
        return out.tolist(), stats

    def spec_generate(self, prompts, n_predict: int, draft_max: int = 4, ngram: int = 3):
        """Greedy speculative decoding by prompt lookup (drafts from each sequence's own context,
        one verify chunk per micro-batch per round); output equals generate() at temp 0."""
        flat, lens = self._flat(prompts)
        out = np.full((len(prompts), n_predict), -1, np.int32)
        stats = N.jcall(N.lib().mp_engine_spec_generate, self._h, flat.ctypes.data, lens.ctypes.data, len(prompts),
                        n_predict, draft_max, ngram, out.ctypes.data, what="spec_generate")
        return out.tolist(), stats

    def start(self, prompts):
        flat, lens = self._flat(prompts)
        self._n_seq = len(prompts)
        N.check(N.lib().mp_engine_start(self._h, flat.ctypes.data, lens.ctypes.data, len(prompts)), "start")

    def admit(self, slots, prompts):
        """Continuous batching: between decode rounds, prefill `prompts` into the idle sequence slots
        `slots` (slot = micro-batch * mb_size + row); the other slots keep generating."""
        flat, lens = self._flat(prompts)
        sl = np.asarray(slots, np.int32)
        N.check(N.lib().mp_engine_admit(self._h, sl.ctypes.data, flat.ctypes.data, lens.ctypes.data, len(prompts)),
                "admit")
        self._n_seq = self.n_seq_cap

    def kv_stats(self):
        """Live paged-KV numbers: pool pages, free pages (the `info` dict is a load-time snapshot)."""
        j = N.jcall(N.lib().mp_engine_info, self._h, what="engine info")
        return {"kv_pages": j["kv_pages"], "kv_free_pages": j["kv_free_pages"]}

    def release(self, slot: int):
        """Mark a slot idle (its sequence is finished); it can be admitted again."""
        N.check(N.lib().mp_engine_release(self._h, int(slot)), "release")

    def decode(self, k: int):
        return N.jcall(N.lib().mp_engine_decode, self._h, k, what="decode")

    def tokens(self, cap: int = 4096):
        out = np.full((self._n_seq, cap), -1, np.int32)
        n = N.check(N.lib().mp_engine_tokens(self._h, out.ctypes.data, self._n_seq, cap), "tokens")
        return [[t for t in row if t >= 0] for row in out[:, :n].tolist()]

    def bench(self, prompt_len: int, warmup: int, steps: int):
        return N.jcall(N.lib().mp_engine_bench, self._h, prompt_len, warmup, steps, what="bench")

    def health(self) -> dict:
        """Per-stage heartbeat (items done), link byte counters, ok=False after a pipeline fault."""
        return N.jcall(N.lib().mp_engine_health, self._h, what="engine health")

    def save_state(self, path: str) -> dict:
        """Checkpoint a running generation: every owned stage's KV shard (used positions only),
        decode inputs and sampler step under `path`/, plus the sequences in session.json."""
        return N.jcall(N.lib().mp_engine_save_state, self._h, N.cstr(path), what="save_state")

    def load_state(self, path: str) -> dict:
        """Resume a generation saved by save_state (same model, partition and micro-batch shape);
        decode() then continues exactly where the saved engine stopped."""
        r = N.jcall(N.lib().mp_engine_load_state, self._h, N.cstr(path), what="load_state")
        self._n_seq = r["sequences"]
        return r

    def trace(self, on: bool = True):
        N.check(N.lib().mp_engine_trace(self._h, int(on), None), "trace")

    def write_trace(self, path: str):
        """Chrome-trace JSON (chrome://tracing, Perfetto) of compute/send/recv spans per stage."""
        N.check(N.lib().mp_engine_trace(self._h, 1, N.cstr(path)), "write trace")

    def logits(self, rows: int = 1, vocab: int | None = None):
        vocab = vocab or self.info["model"]["vocab"]
        out = np.zeros((rows, vocab), np.float32)
        N.check(N.lib().mp_engine_logits(self._h, 0, out.ctypes.data, rows), "logits")
        return out


def device_probe(device: int = 0) -> dict:
    """Halda-style device profile (probe.h): measured HBM read and Q4_K decode-GEMV bandwidth of a
    GPU (device < 0: host memcpy bandwidth, the CPU backend's speed)."""
    out = (ctypes.c_double * 2)()
    N.check(N.lib().mp_device_probe(int(device), out), "device probe")
    return {"hbm_read_gbps": out[0], "gemv_gbps": out[1], "speed": out[1] if out[1] > 0 else out[0]}


def rccl_unique_id_hex() -> str:
    buf = (ctypes.c_uint8 * 128)()
    N.check(N.lib().mp_rccl_unique_id(buf), "rccl unique id")
    return bytes(buf).hex()
