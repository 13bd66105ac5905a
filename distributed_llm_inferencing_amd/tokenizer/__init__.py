"""Offline tokenizers (CPU-side).

There is no network and no HF hub cache, so the default is a deterministic byte-level
tokenizer that works for any vocabulary size:
    ids 0..255      the raw UTF-8 bytes
    bos/eos         the model's special ids (skipped by ``decode(skip_special_tokens=True)``)
    other ids       (random-init models sample the whole vocab) render as one printable
                    ASCII character each, so results stay readable text
If a directory with real tokenizer files is given (e.g. the ``tokenizer/`` folder a shard
export writes next to ``shard_<i>/``, reference ``worker/app.py:167-174``), the HF
``tokenizers``/``transformers`` fast tokenizer is loaded from it instead — offline only.
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import List, Optional

_PRINTABLE = [chr(c) for c in range(33, 127)]


class ByteTokenizer:
    kind = "byte"

    def __init__(self, vocab_size: int, bos_token_id: Optional[int] = None,
                 eos_token_id: Optional[int] = None, add_bos: bool = True):
        self.vocab_size = vocab_size
        self.bos_token_id = bos_token_id
        self.eos_token_id = eos_token_id
        self.add_bos = add_bos and bos_token_id is not None and bos_token_id >= 256

    def encode(self, text: str) -> List[int]:
        ids = list(text.encode("utf-8"))
        ids = [i % self.vocab_size for i in ids]
        if self.add_bos:
            ids = [self.bos_token_id] + ids
        return ids

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        special = {self.bos_token_id, self.eos_token_id}
        out = bytearray()
        for i in ids:
            i = int(i)
            if i in special:
                if skip_special_tokens:
                    continue
                out += f"<|{i}|>".encode()
                continue
            if i < 256:
                out.append(i)
            else:
                out += _PRINTABLE[i % len(_PRINTABLE)].encode()
        return out.decode("utf-8", errors="replace")

    def save_pretrained(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, "dli_tokenizer.json"), "w") as f:
            json.dump({"kind": "byte", "vocab_size": self.vocab_size,
                       "bos_token_id": self.bos_token_id, "eos_token_id": self.eos_token_id,
                       "add_bos": self.add_bos}, f, indent=2)


class HFTokenizer:
    kind = "hf"

    def __init__(self, path: str):
        from transformers import AutoTokenizer  # local files only
        self._tok = AutoTokenizer.from_pretrained(path, local_files_only=True)
        self.bos_token_id = self._tok.bos_token_id
        self.eos_token_id = self._tok.eos_token_id
        self.vocab_size = len(self._tok)

    def encode(self, text: str) -> List[int]:
        return list(self._tok(text)["input_ids"])

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        return self._tok.decode(list(ids), skip_special_tokens=skip_special_tokens)

    def save_pretrained(self, path: str) -> None:
        self._tok.save_pretrained(path)


def load_tokenizer(cfg=None, path: Optional[str] = None):
    """Tokenizer for a model config, preferring real tokenizer files under ``path``."""
    if path and Path(path).is_dir():
        p = Path(path) / "dli_tokenizer.json"
        if p.exists():
            d = json.loads(p.read_text())
            return ByteTokenizer(d["vocab_size"], d.get("bos_token_id"), d.get("eos_token_id"),
                                 d.get("add_bos", True))
        if any((Path(path) / f).exists() for f in ("tokenizer.json", "tokenizer_config.json")):
            try:
                return HFTokenizer(path)
            except Exception:  # noqa: BLE001 - fall back to bytes below
                pass
    if cfg is None:
        return ByteTokenizer(256 + 2, 256, 257)
    return ByteTokenizer(cfg.vocab_size, cfg.bos_token_id, cfg.eos_token_id)
