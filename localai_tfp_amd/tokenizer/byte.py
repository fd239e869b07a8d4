"""Byte-level tokenizer for synthetic / random-init checkpoints."""
from __future__ import annotations

LLAMA3_SPECIALS = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>", "<|end_header_id|>",
                   "<|eot_id|>", "<|reserved_special_token_0|>"]

LLAMA3_CHAT_TEMPLATE = (
    "{{ bos_token }}{% for message in messages %}"
    "{{ '<|start_header_id|>' + message['role'] + '<|end_header_id|>\n\n' + message['content'] | trim + '<|eot_id|>' }}"
    "{% endfor %}{% if add_generation_prompt %}{{ '<|start_header_id|>assistant<|end_header_id|>\n\n' }}{% endif %}")


class ByteTokenizer:
    def __init__(self, vocab_size: int = 512, specials=None, chat_template: str | None = LLAMA3_CHAT_TEMPLATE):
        self.specials = list(specials or LLAMA3_SPECIALS)
        self.vocab_size = max(vocab_size, 256 + len(self.specials))
        self.special_ids = {s: 256 + i for i, s in enumerate(self.specials)}
        self.id_to_special = {v: k for k, v in self.special_ids.items()}
        self.bos_token_id = self.special_ids.get("<|begin_of_text|>")
        eos = [self.special_ids[s] for s in ("<|end_of_text|>", "<|eot_id|>") if s in self.special_ids]
        self.eos_token_ids = eos
        self.eos_token_id = eos[0] if eos else None
        self.bos_token = "<|begin_of_text|>"
        self.eos_token = "<|eot_id|>"
        self.chat_template = chat_template
        self.add_bos = True

    def encode(self, text: str, add_special: bool = True, parse_special: bool = True) -> list[int]:
        out = []
        if add_special and self.add_bos and self.bos_token_id is not None and not text.startswith(self.bos_token):
            out.append(self.bos_token_id)
        i = 0
        while i < len(text):
            if parse_special and text[i] == "<":
                for s, sid in self.special_ids.items():
                    if text.startswith(s, i):
                        out.append(sid)
                        i += len(s)
                        break
                else:
                    out.extend(text[i].encode())
                    i += 1
                continue
            out.extend(text[i].encode())
            i += 1
        return out

    def decode(self, ids, skip_special: bool = True) -> str:
        buf = bytearray()
        parts = []
        for t in ids:
            t = int(t)
            if t < 256:
                buf.append(t)
                continue
            if buf:
                parts.append(buf.decode("utf-8", errors="replace"))
                buf = bytearray()
            if t in self.id_to_special:
                if not skip_special:
                    parts.append(self.id_to_special[t])
            else:
                parts.append(f"<t{t}>")  # never produced by encode(); only random-init models sample these
        if buf:
            parts.append(buf.decode("utf-8", errors="replace"))
        return "".join(parts)

    def token_to_piece(self, t: int) -> str:
        return self.decode([t], skip_special=False)


def _byte_token_bytes(self) -> list[bytes]:
    out = [bytes([i]) for i in range(256)]
    out += [b""] * len(self.specials)
    out += [f"<t{i}>".encode() for i in range(len(out), self.vocab_size)]
    return out


ByteTokenizer.token_bytes = _byte_token_bytes
