"""Synthetic tokenizer vocabularies embedded into synthetic GGUFs.

The reference's model (Llama-3.1-8B) uses a byte-level BPE ("gpt2", pre="llama-bpe") read from
GGUF metadata; TinyLlama / Mixtral / stories15M use SentencePiece-style vocabularies ("llama").
No real vocab files are available offline, so we TRAIN small vocabularies with the HF
`tokenizers` library on local text and pad them to the model's vocab size.  The HF tokenizer
object is kept as an independent oracle for the native C++ BPE tokenizer (tests).
"""
from __future__ import annotations

import functools
import glob
import os

from ..utils.gguf import STRING, I32, F32T, U32

LLAMA3_PAT = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}|"
              r" ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")

# llama.cpp token types
T_NORMAL, T_UNKNOWN, T_CONTROL, T_USER, T_UNUSED, T_BYTE = 1, 2, 3, 4, 5, 6


def corpus_lines(max_bytes: int = 600_000):
    """Deterministic local English-ish text: python stdlib sources (docstrings + code)."""
    files = sorted(glob.glob("/usr/lib/python3.10/*.py"))
    out, total = [], 0
    for f in files:
        try:
            with open(f, encoding="utf-8", errors="ignore") as fh:
                t = fh.read()
        except OSError:
            continue
        out.append(t)
        total += len(t)
        if total > max_bytes:
            break
    if not out:  # pragma: no cover - fallback corpus
        out = ["Once upon a time there was a little model that ran on many GPUs. " * 200]
    return out


@functools.lru_cache(maxsize=4)
def train_bpe(n_merges_vocab: int = 3000):
    """Byte-level BPE with the Llama-3 pre-tokenizer regex. Returns the HF Tokenizer."""
    from tokenizers import Tokenizer, models, pre_tokenizers, trainers, decoders, Regex
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(LLAMA3_PAT), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False),
    ])
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=n_merges_vocab, show_progress=False,
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                                  special_tokens=[])
    tok.train_from_iterator(corpus_lines(), trainer)
    return tok


@functools.lru_cache(maxsize=4)
def train_spm_like(n_vocab: int = 3000):
    """SentencePiece-style BPE pieces (U+2581 word boundary). Returns (pieces, scores)."""
    from tokenizers import Tokenizer, models, pre_tokenizers, trainers
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.Metaspace(replacement="▁", prepend_scheme="always")
    trainer = trainers.BpeTrainer(vocab_size=n_vocab, show_progress=False, special_tokens=[])
    tok.train_from_iterator(corpus_lines(), trainer)
    import json
    model = json.loads(tok.to_str())["model"]
    vocab = model["vocab"]            # token -> id (alphabet first, then merges in order)
    merges = model["merges"]
    rank = {}
    for r, m in enumerate(merges):
        a, b = m if isinstance(m, list) else m.split(" ")
        rank.setdefault(a + b, r)
    pieces, scores = [], []
    for t, _ in sorted(vocab.items(), key=lambda kv: kv[1]):
        pieces.append(t)
        scores.append(-float(rank[t]) if t in rank else 0.0)
    return pieces, scores


def bpe_vocab(vocab_size: int):
    """(tokens, token_types, merges, bos_id, eos_id, eot_id) for a gpt2-style vocab."""
    import json
    tok = train_bpe()
    model = json.loads(tok.to_str())["model"]
    vocab = sorted(model["vocab"].items(), key=lambda kv: kv[1])
    tokens = [t for t, _ in vocab]
    merges = [" ".join(m) if isinstance(m, list) else m for m in model["merges"]]
    types = [T_NORMAL] * len(tokens)
    specials = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>", "<|end_header_id|>",
                "<|eot_id|>"]
    n_normal = vocab_size - 256
    assert len(tokens) <= n_normal
    while len(tokens) < n_normal:
        tokens.append(f"<|reserved_filler_{len(tokens)}|>")
        types.append(T_UNUSED)
    for i in range(256):
        tokens.append(specials[i] if i < len(specials) else f"<|reserved_special_token_{i}|>")
        types.append(T_CONTROL)
    bos = n_normal + 0
    eos = n_normal + 1
    eot = n_normal + 4
    return tokens, types, merges, bos, eos, eot


def spm_vocab(vocab_size: int):
    pieces, scores = train_spm_like()
    tokens = ["<unk>", "<s>", "</s>"]
    types = [T_UNKNOWN, T_CONTROL, T_CONTROL]
    sc = [0.0, 0.0, 0.0]
    for b in range(256):
        tokens.append("<0x%02X>" % b)
        types.append(T_BYTE)
        sc.append(0.0)
    seen = set(tokens)
    for p, s in zip(pieces, scores):
        if p in seen:
            continue
        if len(tokens) >= vocab_size:
            break
        seen.add(p)
        tokens.append(p)
        types.append(T_NORMAL)
        sc.append(s)
    assert len(tokens) <= vocab_size
    while len(tokens) < vocab_size:
        tokens.append(f"<unused_{len(tokens)}>")
        types.append(T_UNUSED)
        sc.append(-1e9)
    return tokens, types, sc


def add_tokenizer_kv(w, cfg):
    if cfg.tokenizer == "gpt2":
        tokens, types, merges, bos, eos, eot = bpe_vocab(cfg.vocab)
        w.add("tokenizer.ggml.model", "gpt2")
        w.add("tokenizer.ggml.pre", "qwen2" if cfg.arch == "qwen2" else "llama-bpe")
        w.add("tokenizer.ggml.tokens", tokens, elem_type=STRING)
        w.add("tokenizer.ggml.token_type", types, elem_type=I32)
        w.add("tokenizer.ggml.merges", merges, elem_type=STRING)
        w.add("tokenizer.ggml.bos_token_id", bos, U32)
        w.add("tokenizer.ggml.eos_token_id", eos, U32)
        w.add("tokenizer.ggml.eot_token_id", eot, U32)
        w.add("tokenizer.ggml.add_bos_token", True)
    else:
        tokens, types, scores = spm_vocab(cfg.vocab)
        w.add("tokenizer.ggml.model", "llama")
        w.add("tokenizer.ggml.tokens", tokens, elem_type=STRING)
        w.add("tokenizer.ggml.scores", scores, elem_type=F32T)
        w.add("tokenizer.ggml.token_type", types, elem_type=I32)
        w.add("tokenizer.ggml.bos_token_id", 1, U32)
        w.add("tokenizer.ggml.eos_token_id", 2, U32)
        w.add("tokenizer.ggml.unknown_token_id", 0, U32)
        w.add("tokenizer.ggml.add_bos_token", True)
        w.add("tokenizer.ggml.add_space_prefix", True)
