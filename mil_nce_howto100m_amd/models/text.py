"""Word2vec bag-of-words text tower (``Sentence_Embedding``, ``s3dg.py:148-204``).

``word_embd`` (66250 x 300) is frozen exactly like ``nn.Embedding.from_pretrained``; fc1 is
300->2048 followed by ReLU and a max over the words, fc2 is 2048->512. Unlike the reference,
``word2vec_path=''`` gives a random-init frozen table (the reference joins '' with its
directory and then fails to load it, ``s3dg.py:158, 238``), which the synthetic benchmark needs.

On GPU the embedding gather, fc1, its bias, the ReLU and the max over words run as ONE HIP
MFMA kernel (``ops.hip_ops.text_tower``) over a bf16 copy of the table padded to 320 columns;
it also records the arg-max word for the backward.
"""
from __future__ import annotations

import os
import re
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


class SentenceEmbedding(nn.Module):
    def __init__(self, embd_dim, token_to_word_path="", num_embeddings=66250, word_embedding_dim=300,
                 word2vec_path="", max_words=16, output_dim=2048):
        super().__init__()
        if word2vec_path and os.path.isfile(word2vec_path):
            table = torch.load(word2vec_path, map_location="cpu", weights_only=True)
            self.word_embd = nn.Embedding.from_pretrained(table)
        else:
            self.word_embd = nn.Embedding(num_embeddings, word_embedding_dim)
            self.word_embd.weight.requires_grad_(False)  # frozen, as from_pretrained(freeze=True)
        self.fc1 = nn.Linear(word_embedding_dim, output_dim)
        self.fc2 = nn.Linear(output_dim, embd_dim)
        self.max_words = max_words
        self.word_to_token: Dict[str, int] = {}
        if token_to_word_path and os.path.isfile(token_to_word_path):
            token_to_word = np.load(token_to_word_path, allow_pickle=False)
            for i, t in enumerate(token_to_word):
                self.word_to_token[str(t)] = i + 1  # token id = index + 1; 0 is padding
        self._bf16_table: Optional[torch.Tensor] = None
        self._bf16_key: Optional[tuple] = None

    # --- raw-text tokenisation (s3dg.py:166-194) -----------------------------------------
    @staticmethod
    def _split_text(sentence) -> List[str]:
        return re.findall(r"[\w']+", str(sentence))

    def _words_to_token(self, words: Sequence[str]) -> torch.Tensor:
        ids = [self.word_to_token[w] for w in words if w in self.word_to_token]
        out = torch.zeros(self.max_words, dtype=torch.long)
        if ids:
            ids = ids[: self.max_words]
            out[: len(ids)] = torch.tensor(ids, dtype=torch.long)
        return out

    def words_to_ids(self, sentences) -> torch.Tensor:
        return torch.stack([self._words_to_token(self._split_text(s)) for s in sentences], dim=0)

    # --- forward (s3dg.py:196-204) --------------------------------------------------------
    def _table(self) -> torch.Tensor:
        """bf16, 32-column-padded copy of the frozen table for the fused GPU kernel; rebuilt when
        the table is replaced or modified in place (e.g. ``load_state_dict``)."""
        w = self.word_embd.weight
        key = (w.device, w.data_ptr(), w._version, tuple(w.shape))
        if self._bf16_table is None or self._bf16_key != key:
            from ..ops import hip_ops
            self._bf16_table = hip_ops.text_table_padded(w)
            self._bf16_key = key
        return self._bf16_table

    def forward(self, x, raw_text=False):
        if raw_text:
            x = self.words_to_ids(x).to(self.fc1.weight.device)
        if x.is_cuda and ops.use_hip(x):
            from ..ops import hip_ops
            return hip_ops.text_tower(x, self._table(), self.fc1.weight, self.fc1.bias,
                                      self.fc2.weight, self.fc2.bias)
        with torch.no_grad():
            e = F.embedding(x, self.word_embd.weight)
        h = F.linear(e, self.fc1.weight, self.fc1.bias)
        h = ops.text_relu_max(h)
        return F.linear(h, self.fc2.weight, self.fc2.bias)
