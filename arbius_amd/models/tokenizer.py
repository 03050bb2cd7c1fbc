"""CLIP prompt tokenizer.

With real checkpoint files (``vocab.json`` + ``merges.txt``) the byte-level
CLIP BPE from ``transformers`` is used.  Without them (this sandbox has no
network, BASELINE.json: "synthetic prompts / random-init weights") a
deterministic hashed-word tokenizer with the same id layout is used: BOS
49406, EOS 49407 (also the pad id, as in SD1.5), 77 positions.
"""
from __future__ import annotations

import hashlib
import re
from pathlib import Path
from typing import List, Optional

BOS, EOS, VOCAB, MAX_LEN = 49406, 49407, 49408, 77
_WORD = re.compile(r"[a-z]+|[0-9]|[^\sa-z0-9]+")


class CLIPTokenizer:
    def __init__(self, vocab_dir: Optional[str] = None, max_len: int = MAX_LEN, vocab: int = VOCAB):
        self.max_len = max_len
        self.vocab = vocab
        self._bpe = None
        if vocab_dir and (Path(vocab_dir) / "vocab.json").exists():
            from transformers import CLIPTokenizer as HFTok  # offline, local files only
            self._bpe = HFTok(str(Path(vocab_dir) / "vocab.json"), str(Path(vocab_dir) / "merges.txt"))

    def _hash_ids(self, text: str) -> List[int]:
        ids = []
        span = max(1, min(self.vocab, BOS) - 256)
        for w in _WORD.findall(" ".join(text.lower().split())):
            h = int.from_bytes(hashlib.blake2b(w.encode(), digest_size=8).digest(), "little")
            ids.append(256 + h % span)
        return ids

    def __call__(self, text: str) -> List[int]:
        if self._bpe is not None:
            ids = self._bpe(text, add_special_tokens=False)["input_ids"]
        else:
            ids = self._hash_ids(text)
        bos = min(BOS, self.vocab - 2)
        eos = min(EOS, self.vocab - 1)
        ids = [bos] + ids[: self.max_len - 2] + [eos]
        return ids + [eos] * (self.max_len - len(ids))
