"""CLIP byte-level BPE tokenizer + ``tokenize`` (host-side, init-time only).

Behaviour follows ``PromptSRC/clip/simple_tokenizer.py:62-127`` (vocab 49408,
SOT 49406, EOT 49407, digits one token each) and ``PromptSRC/clip/clip.py:185-221``
(SOT + BPE + EOT, zero-padded to 77, RuntimeError when too long unless truncate).

The merges file (``bpe_simple_vocab_16e6.txt.gz``) is OpenAI's public CLIP vocab; it is
not shipped here. It is looked up at ``$FSP_BPE_VOCAB`` or next to this file (copy it there
once on a box with real datasets); no other location is searched. Without it, a small
word→id table (``bpe_fallback.json``, generated from the vocab by
``tests/golden/make_golden.py``) covers the synthetic prompts used by tests and benchmarks
("X", "a photo of a", "classK."); any other word raises a KeyError that names the file and
the variable.
"""
from __future__ import annotations

import gzip
import html
import json
import os
from functools import lru_cache

import numpy as np

try:
    import regex as _re
except ImportError:  # pragma: no cover - regex is in the image
    _re = None

SOT_TOKEN = 49406
EOT_TOKEN = 49407
CONTEXT_LENGTH = 77

_HERE = os.path.dirname(os.path.abspath(__file__))
_PATTERN = (r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|"""
            r"""[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+""")


def _vocab_candidates():
    env = os.environ.get("FSP_BPE_VOCAB")
    if env:
        yield env
    yield os.path.join(_HERE, "bpe_simple_vocab_16e6.txt.gz")


def find_vocab():
    for p in _vocab_candidates():
        if p and os.path.isfile(p):
            return p
    return None


@lru_cache()
def _byte_alphabet():
    """Map each byte 0..255 to a printable unicode char (GPT-2/CLIP byte-level scheme).

    Iteration order matters: the vocab lists the printable bytes first (in byte order),
    then the remapped control/space bytes (256+n), exactly as the CLIP vocab does."""
    printable = sorted(set(range(0x21, 0x7F)) | set(range(0xA1, 0xAD)) | set(range(0xAE, 0x100)))
    table = {b: chr(b) for b in printable}
    extra = 0
    for b in range(256):
        if b not in table:
            table[b] = chr(256 + extra)
            extra += 1
    return table


def _clean(text: str) -> str:
    # ftfy.fix_text is the identity on the plain-ASCII class names used here; it is
    # applied when ftfy is importable (simple_tokenizer.py:50-53).
    try:  # pragma: no cover - ftfy absent in the image
        import ftfy
        text = ftfy.fix_text(text)
    except ImportError:
        pass
    text = html.unescape(html.unescape(text)).strip()
    text = " ".join(text.split())
    return text.lower()


class BPETokenizer:
    def __init__(self, vocab_path: str | None = None):
        self.vocab_path = vocab_path or find_vocab()
        self._fallback = None
        if self.vocab_path is None:
            with open(os.path.join(_HERE, "bpe_fallback.json")) as f:
                self._fallback = json.load(f)
            self.encoder = None
            return
        with gzip.open(self.vocab_path) as f:
            lines = f.read().decode("utf-8").split("\n")
        merges = [tuple(l.split()) for l in lines[1:49152 - 256 - 2 + 1]]
        alphabet = list(_byte_alphabet().values())
        tokens = alphabet + [c + "</w>" for c in alphabet] + ["".join(m) for m in merges]
        tokens += ["<|startoftext|>", "<|endoftext|>"]
        self.encoder = {t: i for i, t in enumerate(tokens)}
        self.ranks = {m: i for i, m in enumerate(merges)}
        self._cache = {}

    def _merge_word(self, word: str):
        if word in self._cache:
            return self._cache[word]
        parts = list(word[:-1]) + [word[-1] + "</w>"]
        while len(parts) > 1:
            best, best_rank = None, None
            for i in range(len(parts) - 1):
                r = self.ranks.get((parts[i], parts[i + 1]))
                if r is not None and (best_rank is None or r < best_rank):
                    best, best_rank = (parts[i], parts[i + 1]), r
            if best is None:
                break
            merged, i = [], 0
            while i < len(parts):
                if i + 1 < len(parts) and parts[i] == best[0] and parts[i + 1] == best[1]:
                    merged.append(best[0] + best[1])
                    i += 2
                else:
                    merged.append(parts[i])
                    i += 1
            parts = merged
        self._cache[word] = parts
        return parts

    def words(self, text: str):
        if _re is None:  # pragma: no cover
            raise RuntimeError("the 'regex' module is required for tokenization")
        return _re.findall(_re.compile(_PATTERN, _re.IGNORECASE), _clean(text))

    def encode_word(self, word: str):
        if self.encoder is None:
            if word not in self._fallback:
                raise KeyError(f"CLIP BPE vocab not found and '{word}' is not in the synthetic-name "
                               f"fallback table: set $FSP_BPE_VOCAB to the path of "
                               f"bpe_simple_vocab_16e6.txt.gz (or copy it to {_HERE})")
            return list(self._fallback[word])
        ab = _byte_alphabet()
        w = "".join(ab[b] for b in word.encode("utf-8"))
        return [self.encoder[p] for p in self._merge_word(w)]

    def encode(self, text: str):
        out = []
        for w in self.words(text):
            out += self.encode_word(w)
        return out


@lru_cache()
def default_tokenizer() -> BPETokenizer:
    return BPETokenizer()


def tokenize(texts, context_length: int = CONTEXT_LENGTH, truncate: bool = False) -> np.ndarray:
    """int64 [len(texts), context_length] token ids, SOT ... EOT then zeros."""
    if isinstance(texts, str):
        texts = [texts]
    tok = default_tokenizer()
    out = np.zeros((len(texts), context_length), dtype=np.int64)
    for i, t in enumerate(texts):
        ids = [SOT_TOKEN] + tok.encode(t) + [EOT_TOKEN]
        if len(ids) > context_length:
            if not truncate:
                raise RuntimeError(f"Input {t} is too long for context length {context_length}")
            ids = ids[:context_length]
            ids[-1] = EOT_TOKEN
        out[i, :len(ids)] = ids
    return out
