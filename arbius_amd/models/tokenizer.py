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


# where checkpoint directories keep their tokenizer files: the root, the diffusers ``tokenizer/``
# folder, or a per-tower folder of a multi-encoder pipeline (Kandinsky 2: XLM-R in tokenizer/,
# CLIP in the prior checkout's prior/tokenizer/)
TOKENIZER_SUBDIRS = ("", "tokenizer", "clip_tokenizer", "tokenizer_clip", "prior/tokenizer", "text_encoder")


def find_file(root: Optional[str], name: str, subdirs=TOKENIZER_SUBDIRS) -> Optional[Path]:
    """First ``root/<subdir>/name`` that exists (tokenizer auto-discovery from a weights dir)."""
    if not root:
        return None
    for sub in subdirs:
        f = Path(root) / sub / name
        if f.is_file():
            return f
    return None


class CLIPTokenizer:
    """``vocab_dir``: a directory holding ``vocab.json`` + ``merges.txt`` directly or in one of
    ``TOKENIZER_SUBDIRS`` (so a pipeline can be handed its weights dir)."""

    def __init__(self, vocab_dir: Optional[str] = None, max_len: int = MAX_LEN, vocab: int = VOCAB):
        self.max_len = max_len
        self.vocab = vocab
        self._bpe = None
        self.source = "hashed-words"
        vj = find_file(vocab_dir, "vocab.json")
        if vj is not None and (vj.parent / "merges.txt").is_file():
            from transformers import CLIPTokenizer as HFTok  # offline, local files only
            self._bpe = HFTok(str(vj), str(vj.parent / "merges.txt"))
            self.source = str(vj.parent)

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
