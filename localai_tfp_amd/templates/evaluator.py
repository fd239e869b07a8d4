"""Prompt templating (reference: pkg/templates/evaluator.go:17-295, cache.go:23-184).

`TemplateMessages` turns an OpenAI message list into the model prompt: each message through
the `chat_message` template (Go or Jinja), joined (default "\n"), then wrapped by the `chat`
(or `function` when tools are active) template. Template strings may also name a
`<models>/<name>.tmpl` file. With `template.use_tokenizer_template` the whole conversation goes
through the model's own Jinja chat template instead (the GGUF `tokenizer.chat_template`).
"""
from __future__ import annotations

import json
import logging
import os

from . import gotemplate
from .chat import render_jinja

log = logging.getLogger("localai_tfp_amd.templates")

CHAT, CHAT_MESSAGE, COMPLETION, EDIT, FUNCTIONS = range(5)


class Evaluator:
    def __init__(self, model_path: str = ""):
        self.model_path = model_path

    # ---------------------------------------------------------------- template resolution
    def _resolve(self, name_or_src: str) -> str:
        """A template value may be inline text or the basename of a .tmpl file in the models dir."""
        if not name_or_src:
            return ""
        if self.model_path and "{{" not in name_or_src and "{%" not in name_or_src:
            cand = os.path.join(self.model_path, name_or_src if name_or_src.endswith(".tmpl") else name_or_src + ".tmpl")
            if os.path.isfile(cand) and os.path.realpath(cand).startswith(os.path.realpath(self.model_path)):
                with open(cand, encoding="utf-8") as f:
                    return f.read()
        return name_or_src

    def evaluate_for_prompt(self, kind: int, cfg, data: dict) -> str:
        tpl = ""
        model_file_tmpl = self._resolve(cfg.parameters.model) if cfg.parameters.model else ""
        if model_file_tmpl and model_file_tmpl != cfg.parameters.model:
            tpl = model_file_tmpl
        t = cfg.template
        pick = {COMPLETION: t.completion, EDIT: t.edit, CHAT: t.chat, FUNCTIONS: t.function}.get(kind, "")
        if pick:
            tpl = self._resolve(pick)
        if not tpl:
            return data.get("Input", "")
        if t.jinja_template:
            return render_jinja(tpl, [], add_generation_prompt=True, system_prompt=data.get("SystemPrompt", ""),
                                content=data.get("Input", ""))
        return gotemplate.render(tpl, data)

    # ---------------------------------------------------------------- chat
    def template_messages(self, messages: list[dict], cfg, funcs: list | None, should_use_fn: bool) -> str:
        t = cfg.template
        roles = cfg.roles or {}
        if t.jinja_template and t.chat_message:
            try:
                msgs = []
                for i, m in enumerate(messages):
                    fc = m.get("tool_calls") or m.get("function_call")
                    msgs.append({"role": m.get("role", ""), "content": m.get("string_content", ""),
                                 "function_call": fc, "name": m.get("name", "")})
                return render_jinja(self._resolve(t.chat_message), msgs, add_generation_prompt=True,
                                    tools=funcs or None, system_prompt=cfg.system_prompt)
            except Exception as ex:
                log.warning("jinja chat template failed, falling back: %s", ex)
        suppress_sys = False
        parts = []
        n = len(messages)
        for idx, m in enumerate(messages):
            role = m.get("role", "")
            fcall = m.get("tool_calls") or m.get("function_call")
            if fcall and role == "assistant" and roles.get("assistant_function_call"):
                role = "assistant_function_call"
            r = roles.get(role, "")
            content_str = m.get("string_content", "") or ""
            content_exists = m.get("content") is not None and content_str != ""
            content = ""
            if t.chat_message:
                data = {
                    "SystemPrompt": cfg.system_prompt, "Role": r, "RoleName": role, "Content": content_str,
                    "FunctionCall": fcall, "FunctionName": m.get("name", ""), "LastMessage": idx == n - 1,
                    "Function": bool(cfg.grammar) and idx == n - 1, "MessageIndex": idx,
                }
                try:
                    content = gotemplate.render(self._resolve(t.chat_message), data)
                    if content == "":
                        log.warning("chat_message template produced blank output for message %d; skipping", idx)
                        continue
                except Exception as ex:
                    log.error("chat_message template failed for message %d: %s", idx, ex)
                    content = ""
            if content == "":
                if r:
                    if content_exists:
                        content = r + content_str
                    if fcall is not None:
                        j = json.dumps(fcall, separators=(",", ":"))
                        content = (content + "\n" + r + " " + j) if content_exists else (r + " " + j)
                else:
                    if content_exists:
                        content = content_str
                    if fcall is not None:
                        j = json.dumps(fcall, separators=(",", ":"))
                        content = (content + "\n" + j) if content_exists else j
                if content_exists and role == "system":
                    suppress_sys = True
            parts.append(content)
        join = "\n" if t.join_chat_messages_by_character is None else t.join_chat_messages_by_character
        pred = join.join(parts)
        kind = FUNCTIONS if (t.function and should_use_fn) else CHAT
        try:
            pred = self.evaluate_for_prompt(kind, cfg, {
                "SystemPrompt": cfg.system_prompt, "SuppressSystemPrompt": suppress_sys, "Input": pred,
                "Functions": [f if isinstance(f, dict) else vars(f) for f in (funcs or [])], "Instruction": "",
                "MessageIndex": 0,
            })
        except Exception as ex:
            log.debug("prompt template failed: %s", ex)
        return pred
