"""Jinja chat templates embedded in model files (`tokenizer.chat_template`), rendered in a sandbox.

The reference falls back to the GGUF's raw Jinja template when no Go template matches
(core/config/gguf.go:255-296, `UseTokenizerTemplate`) and renders Jinja via gonja
(pkg/templates/cache.go:123). Same behaviour here with jinja2's SandboxedEnvironment and the
HF-compatible globals (raise_exception, strftime_now) templates expect.
"""
from __future__ import annotations

import datetime
import functools

from jinja2 import StrictUndefined, Undefined
from jinja2.sandbox import ImmutableSandboxedEnvironment


def _raise(msg):
    raise ValueError(msg)


@functools.lru_cache(maxsize=64)
def _compile(src: str):
    env = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True, undefined=Undefined)
    env.globals["raise_exception"] = _raise
    env.globals["strftime_now"] = lambda fmt: datetime.datetime.now().strftime(fmt)
    env.filters["tojson"] = __import__("json").dumps
    return env.from_string(src)


def render_jinja(src: str, messages, add_generation_prompt: bool = True, bos_token: str = "",
                 eos_token: str = "", tools=None, **extra) -> str:
    tpl = _compile(src)
    return tpl.render(messages=messages, add_generation_prompt=add_generation_prompt, bos_token=bos_token,
                      eos_token=eos_token, tools=tools, **extra)


def render_chat(messages, tok, add_generation_prompt: bool = True, tools=None) -> str:
    src = getattr(tok, "chat_template", None)
    if not src:
        # plain fallback: "role: content" lines
        s = "".join(f"{m['role']}: {m['content']}\n" for m in messages)
        return s + ("assistant: " if add_generation_prompt else "")
    return render_jinja(src, messages, add_generation_prompt, getattr(tok, "bos_token", ""),
                        getattr(tok, "eos_token", ""), tools)
