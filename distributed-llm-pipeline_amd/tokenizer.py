"""Python handle on the native GGUF tokenizer (csrc/runtime/tokenizer.cpp): byte-level BPE
(gpt2 / Llama-3 pre-tokenizer) and SentencePiece-style (llama) vocabularies read from GGUF
metadata (reference: llama.cpp's llama-vocab)."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N


class Tokenizer:
    def __init__(self, gguf_path: str):
        L = N.lib()
        h = L.mp_tok_open(N.cstr(gguf_path))
        if not h:
            N.check(None, "tokenizer open")
        self._h = ctypes.c_void_p(h)
        info = np.zeros(4, np.int32)
        N.check(L.mp_tok_info(self._h, info.ctypes.data), "tokenizer info")
        self.n_vocab, self.bos, self.eos, self.eot = (int(v) for v in info)

    def close(self):
        if getattr(self, "_h", None):
            N.lib().mp_tok_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def encode(self, text: str, add_bos: bool = False, parse_special: bool = True) -> list[int]:
        b = text.encode("utf-8")
        cap = len(b) + 16
        out = np.zeros(cap, np.int32)
        n = N.lib().mp_tok_encode(self._h, b, int(add_bos), int(parse_special), out.ctypes.data, cap)
        if n < 0:
            N.check(None, "encode")
        if n > cap:   # pragma: no cover - cannot happen for byte-level vocabularies
            out = np.zeros(n, np.int32)
            N.lib().mp_tok_encode(self._h, b, int(add_bos), int(parse_special), out.ctypes.data, n)
        return out[:n].tolist()

    def decode(self, ids) -> str:
        ids = np.asarray(ids, np.int32)
        cap = 16 * len(ids) + 64
        buf = ctypes.create_string_buffer(cap)
        n = N.lib().mp_tok_decode(self._h, ids.ctypes.data, len(ids), buf, cap)
        if n < 0:
            N.check(None, "decode")
        return buf.raw[:n].decode("utf-8", errors="replace")

    def piece(self, tid: int) -> bytes:
        buf = ctypes.create_string_buffer(256)
        n = N.lib().mp_tok_piece(self._h, int(tid), buf, 256)
        return buf.raw[:n]

    @staticmethod
    def pretokenize(text: str, pre: str = "llama-bpe") -> list[str]:
        """The native pre-tokenizer split (regex-free implementation): "llama-bpe" (Llama-3, numbers
        in groups of up to 3 digits) or "qwen2" (single digits)."""
        r = N.lib().mp_tok_pretokenize(text.encode("utf-8"), 1 if pre == "qwen2" else 3)
        return r.decode("utf-8").split("\x1f")[:-1]
