"""Prompt weighting for the CLIP-conditioned pipelines (the reference's diffusers backend enables Compel with
COMPEL=1, backend/python/diffusers/backend.py:40-46,230-236).

Syntax (Compel, plus the common A1111 form):
  ``(a red car)1.3``  ``(a red car)++``  ``car+`` / ``car--``   weight 1.1^(#+) / 0.9^(#-), or the number
  ``(a red car:1.3)``                                             A1111-style explicit weight
Weights multiply per token; nesting multiplies. Application (Compel-style, parity unpinned — Compel is not
available here): the prompt is encoded once with its words unweighted and once empty; each token's hidden
state becomes  empty + w * (prompt - empty),  so weight 1 reproduces the plain embedding exactly.
"""
from __future__ import annotations

import re

_NUM = r"[0-9]*\.?[0-9]+"


def parse(prompt: str) -> list[tuple[str, float]]:
    """-> [(text, weight)] chunks in order (weight 1.0 for plain text)."""
    out: list[tuple[str, float]] = []
    stack: list[list[tuple[str, float]]] = [[]]
    i, n = 0, len(prompt)
    while i < n:
        ch = prompt[i]
        if ch == "(":
            stack.append([])
            i += 1
            continue
        if ch == ")" and len(stack) > 1:
            j = i + 1
            m = re.match(_NUM, prompt[j:])
            if m:
                w = float(m.group(0))
                j += m.end()
            else:
                k = j
                while k < n and prompt[k] in "+-":
                    k += 1
                sig = prompt[j:k]
                w = 1.1 ** sig.count("+") * 0.9 ** sig.count("-") if sig else 1.1
                j = k
            inner = stack.pop()
            stack[-1].extend((t, x * w) for t, x in inner)
            i = j
            continue
        # plain run up to the next paren
        j = i
        while j < n and prompt[j] not in "()":
            j += 1
        run = prompt[i:j]
        # A1111 "(text:1.3)": a trailing ":<num>" right before the closing paren
        m = re.search(r":(" + _NUM + r")\s*$", run)
        if m and j < n and prompt[j] == ")" and len(stack) > 1:
            stack[-1].append((run[:m.start()], float(m.group(1))))
            # the closing paren then applies weight 1 (the number was consumed here)
            inner = stack.pop()
            stack[-1].extend(inner)
            i = j + 1
            continue
        for word in re.split(r"(\s+)", run):
            if not word:
                continue
            wm = re.fullmatch(r"(.*?[^+-])([+-]+)", word)
            if wm and not word.isspace():
                sig = wm.group(2)
                stack[-1].append((wm.group(1), 1.1 ** sig.count("+") * 0.9 ** sig.count("-")))
            else:
                stack[-1].append((word, 1.0))
        i = j
    while len(stack) > 1:  # unbalanced "(": treat as plain text
        inner = stack.pop()
        stack[-1].extend(inner)
    for t, w in stack[0]:
        if out and out[-1][1] == w:
            out[-1] = (out[-1][0] + t, w)
        else:
            out.append((t, w))
    return [(t, w) for t, w in out if t.strip()] or [("", 1.0)]


def weighted_ids(tok, prompt: str) -> tuple[list[int], list[float]]:
    """CLIP ids (bos, tokens, eos, pad to max_len) and one weight per position (1.0 on specials / padding)."""
    ids, ws = [tok.bos], [1.0]
    for text, w in parse(prompt):
        t = tok.encode(text)
        ids += t
        ws += [w] * len(t)
    ids, ws = ids[: tok.max_len - 1] + [tok.eos], ws[: tok.max_len - 1] + [1.0]
    pad = tok.max_len - len(ids)
    return ids + [tok.pad] * pad, ws + [1.0] * pad


def has_weights(prompt: str) -> bool:
    return any(w != 1.0 for _, w in parse(prompt))


def has_syntax(prompt: str) -> bool:
    """Weighting syntax present (even weight 1): the prompt must go through the parser."""
    c = parse(prompt)
    return any(w != 1.0 for _, w in c) or "".join(t for t, _ in c).strip() != prompt.strip()


def apply(hidden, empty_hidden, weights):
    """hidden / empty_hidden [S, D] (one prompt) -> empty + w * (hidden - empty), w per position."""
    import torch
    w = torch.tensor(weights, dtype=hidden.dtype, device=hidden.device)[:, None]
    return empty_hidden + w * (hidden - empty_hidden)
