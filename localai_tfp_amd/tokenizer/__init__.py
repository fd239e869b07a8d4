"""Tokenizers for the LLM worker.

* :class:`ByteTokenizer` — byte-level tokenizer used by synthetic checkpoints (ids 0..255 are raw
  bytes; special tokens follow; the remaining ids up to the model's vocab are never produced by
  `encode` but decode to a short placeholder so random-init models still stream text).
* :func:`from_gguf` — builds the tokenizer embedded in a GGUF file (``tokenizer.ggml.*``):
  byte-level BPE (gpt2/llama-bpe, Llama-3, Qwen2) through HF ``tokenizers`` and SentencePiece-style
  (llama/mistral "llama" model) through :mod:`.spm`. See tokenizer/gguf.py.
"""
from __future__ import annotations

from .byte import ByteTokenizer  # noqa: F401
from .gguf import from_gguf  # noqa: F401
from .hf import from_hf_dir  # noqa: F401
