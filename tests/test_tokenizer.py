"""Native tokenizer (csrc/runtime/tokenizer.cpp) against independent oracles (CPU):
  * BPE: the HF `tokenizers` tokenizer the GGUF vocabulary was trained with (same ids), and the
    `regex`-module Llama-3 pre-tokenizer pattern for the hand-written splitter;
  * SPM: a direct Python transcription of SentencePiece-style bigram merging by score with byte
    fallback (llama.cpp's llm_tokenizer_spm behaviour; parity unpinned against sentencepiece
    itself since no real .model file is available offline)."""
import pytest

from conftest import make_model

TEXTS = [
    "Once upon a time there was a little GPU.",
    "def f(x):\n    return x ** 2  # square\n",
    "I'll say it's   done, we'd've known!",
    "numbers 1234567 and 3.14159, 2024-01-30",
    "unicode: héllo wörld — naïve café, 日本語テキスト, Привет мир 🚀🔥",
    "tabs\tand\nnew\n\nlines   \n  trailing spaces   ",
    "   leading spaces",
    "",
    "a",
    "!!!???...",
    "MiXeD CaSe WORDS and 'quotes' \"double\"",
]


@pytest.fixture(scope="module")
def bpe(native, model_dir):
    from mipipe.tokenizer import Tokenizer
    path, cfg = make_model(model_dir, "tiny-l3", "Q8_0")
    return Tokenizer(path)


@pytest.fixture(scope="module")
def spm(native, model_dir):
    from mipipe.tokenizer import Tokenizer
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    return Tokenizer(path)


def test_pretokenizer_matches_regex(native):
    import regex
    from mipipe.models.tokenizer_data import LLAMA3_PAT
    from mipipe.tokenizer import Tokenizer
    pat = regex.compile(LLAMA3_PAT)
    for t in TEXTS + ["x's y'T Z'Ll", "  \n\n  a", "123456789012", "😀😀 a😀b"]:
        assert Tokenizer.pretokenize(t) == pat.findall(t), t
    # Qwen2's pre-tokenizer differs only in splitting numbers into single digits
    qpat = regex.compile(LLAMA3_PAT.replace(r"\p{N}{1,3}", r"\p{N}"))
    assert qpat.pattern != pat.pattern
    for t in TEXTS + ["123456789012 and 3.14159", "x1y22z333"]:
        assert Tokenizer.pretokenize(t, "qwen2") == qpat.findall(t), t


def test_bpe_matches_hf_tokenizers(bpe):
    from mipipe.models.tokenizer_data import train_bpe
    hf = train_bpe()
    for t in TEXTS:
        assert bpe.encode(t, add_bos=False, parse_special=False) == hf.encode(t).ids, t


def test_bpe_roundtrip_and_specials(bpe):
    for t in TEXTS:
        assert bpe.decode(bpe.encode(t)) == t
    ids = bpe.encode("<|begin_of_text|>hello<|eot_id|>", parse_special=True)
    assert ids[0] == bpe.bos and ids[-1] == bpe.eot
    assert bpe.encode("hello", add_bos=True)[0] == bpe.bos
    # without special parsing the marker is plain text
    assert bpe.bos not in bpe.encode("<|begin_of_text|>", parse_special=False)


def _spm_reference(text, tokens, scores):
    """SentencePiece-style encoding: '▁' for spaces (+ prefix), bigram merges by best score
    (leftmost on ties), unknown pieces fall back to <0xXX> byte tokens."""
    vocab = {t: i for i, t in enumerate(tokens)}
    s = "▁" + text.replace(" ", "▁")
    syms = list(s)
    while True:
        best, best_i = None, -1
        for i in range(len(syms) - 1):
            m = syms[i] + syms[i + 1]
            if m in vocab and (best is None or scores[vocab[m]] > best):
                best, best_i = scores[vocab[m]], i
        if best_i < 0:
            break
        syms[best_i:best_i + 2] = [syms[best_i] + syms[best_i + 1]]
    out = []
    for sym in syms:
        if sym in vocab:
            out.append(vocab[sym])
        else:
            out.extend(vocab["<0x%02X>" % b] for b in sym.encode("utf-8"))
    return out


def test_spm_matches_reference(spm, model_dir):
    from mipipe.models.config import CONFIGS
    from mipipe.models.tokenizer_data import spm_vocab
    tokens, types, scores = spm_vocab(CONFIGS["tiny-gqa"].vocab)
    for t in [x for x in TEXTS if x and not x.startswith(" ")] + ["hello world", "the quick brown fox"]:
        assert spm.encode(t, add_bos=False, parse_special=False) == _spm_reference(t, tokens, scores), t


def test_spm_roundtrip(spm):
    for t in ["hello world", "Once upon a time", "日本語 and bytes 🚀", "multiple   spaces"]:
        ids = spm.encode(t, add_bos=True)
        assert ids[0] == spm.bos
        assert spm.decode(ids[1:]).lstrip(" ") == t.lstrip(" ")
