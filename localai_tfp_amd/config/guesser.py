"""Default guessing from the model file (reference: core/config/gguf.go:149-296, guesser.go:7-34).

For a GGUF model with no template in its YAML, the architecture / special tokens select a chat
family and its Go-template prompt format + stop words; when the family is unknown the GGUF's own
Jinja `tokenizer.chat_template` is used instead (template.use_tokenizer_template). Context size
defaults to the trained context capped by LOCALAI_DEFAULT_CONTEXT (default 4096, the reference
worker's default `context_size`, core/backend/options.go:102-105). Set LOCALAI_DISABLE_GUESSING
to turn it off.
"""
from __future__ import annotations

import logging
import os

log = logging.getLogger("localai_tfp_amd.config")

# family -> (template fields, stop words, repeat_penalty)
FAMILIES: dict[str, dict] = {
    "llama3": {
        "stop": ["<|eot_id|>"],
        "template": {
            "chat": "<|begin_of_text|>{{.Input }}\n<|start_header_id|>assistant<|end_header_id|>",
            "chat_message": "<|start_header_id|>{{ .RoleName }}<|end_header_id|>\n\n{{.Content }}<|eot_id|>",
        },
    },
    "chatml": {
        "stop": ["<|im_end|>", "<dummy32000>", "</s>"],
        "template": {
            "chat": "{{.Input -}}\n<|im_start|>assistant",
            "chat_message": (
                "<|im_start|>{{ .RoleName }}\n"
                "{{ if .FunctionCall -}}Function call:\n{{ else if eq .RoleName \"tool\" -}}Function response:\n{{ end -}}"
                "{{ if .Content -}}{{.Content }}\n{{ end -}}"
                "{{ if .FunctionCall -}}{{toJson .FunctionCall}}\n{{ end -}}<|im_end|>"),
            "function": (
                "<|im_start|>system\nYou are a function calling AI model. Call one or more of the following "
                "functions when they help answer the user. Do not guess argument values.\n"
                "{{range .Functions}}{'type': 'function', 'function': {'name': '{{.Name}}', "
                "'description': '{{.Description}}', 'parameters': {{toJson .Parameters}} }}\n{{end}}"
                "Return a JSON object with the function name and its arguments for each call.\n<|im_end|>\n"
                "{{.Input -}}\n<|im_start|>assistant"),
        },
    },
    "gemma": {
        "stop": ["<|im_end|>", "<end_of_turn>", "<start_of_turn>"],
        "repeat_penalty": 1.0,
        "template": {
            "chat": "{{.Input }}\n<start_of_turn>model\n",
            "chat_message": ("<start_of_turn>{{if eq .RoleName \"assistant\" }}model{{else}}{{ .RoleName }}{{end}}\n"
                             "{{ if .Content -}}{{.Content -}}\n{{ end -}}<end_of_turn>"),
            "completion": "{{.Input}}",
        },
    },
    "phi3": {
        "stop": ["<|end|>", "<|endoftext|>"],
        "template": {
            "chat": "{{.Input}}\n<|assistant|>",
            "chat_message": "<|{{ .RoleName }}|>\n{{.Content}}<|end|>",
            "completion": "{{.Input}}",
        },
    },
    "mistral": {
        "stop": ["</s>", "[/TOOL_CALLS]", "<|im_end|>"],
        "template": {
            "chat": "{{.Input -}}",
            "chat_message": ("{{if eq .RoleName \"user\" -}}[INST] {{.Content }} [/INST]"
                             "{{- else if .FunctionCall -}}[TOOL_CALLS] {{toJson .FunctionCall}} [/TOOL_CALLS]"
                             "{{- else if eq .RoleName \"tool\" -}}[TOOL_RESULTS] {{.Content}} [/TOOL_RESULTS]"
                             "{{- else -}}{{ .Content -}}{{ end -}}"),
            "function": ("[AVAILABLE_TOOLS] [{{range .Functions}}{\"type\": \"function\", \"function\": "
                         "{\"name\": \"{{.Name}}\", \"description\": \"{{.Description}}\", \"parameters\": "
                         "{{toJson .Parameters}} }}{{end}} ] [/AVAILABLE_TOOLS]{{.Input }}"),
        },
    },
    "deepseek2": {
        "stop": ["<｜end▁of▁sentence｜>"],
        "template": {
            "chat": "{{.Input -}}\nAssistant: ",
            "chat_message": ("{{if eq .RoleName \"user\" -}}User: {{.Content }}\n{{ end -}}"
                             "{{if eq .RoleName \"assistant\" -}}Assistant: {{.Content}}<｜end▁of▁sentence｜>{{end}}"
                             "{{if eq .RoleName \"system\" -}}{{.Content}}\n{{end -}}"),
        },
    },
    "command-r": {
        "stop": ["<|END_OF_TURN_TOKEN|>"],
        "template": {
            "chat": "{{.Input -}}<|START_OF_TURN_TOKEN|><|CHATBOT_TOKEN|>",
            "chat_message": ("{{if eq .RoleName \"user\" -}}<|START_OF_TURN_TOKEN|><|USER_TOKEN|>{{.Content}}<|END_OF_TURN_TOKEN|>"
                             "{{- else if eq .RoleName \"system\" -}}<|START_OF_TURN_TOKEN|><|SYSTEM_TOKEN|>{{.Content}}<|END_OF_TURN_TOKEN|>"
                             "{{- else if eq .RoleName \"assistant\" -}}<|START_OF_TURN_TOKEN|><|CHATBOT_TOKEN|>{{.Content}}<|END_OF_TURN_TOKEN|>"
                             "{{- else if eq .RoleName \"tool\" -}}<|START_OF_TURN_TOKEN|><|SYSTEM_TOKEN|>{{.Content}}<|END_OF_TURN_TOKEN|>"
                             "{{- end -}}"),
        },
    },
}


def identify_family(md: dict) -> str | None:
    arch = str(md.get("general.architecture", ""))
    tmpl = str(md.get("tokenizer.chat_template", "") or "")
    toks = md.get("tokenizer.ggml.tokens") or []
    tokset = set(toks[-512:]) | set(toks[:512]) if toks else set()
    if "<|eot_id|>" in tokset or "<|start_header_id|>" in tmpl:
        return "llama3"
    if arch in ("gemma", "gemma2", "gemma3") or "<start_of_turn>" in tmpl:
        return "gemma"
    if arch == "phi3" or "<|assistant|>" in tmpl:
        return "phi3"
    if arch in ("command-r", "cohere2"):
        return "command-r"
    if arch == "deepseek2":
        return "deepseek2"
    if "<|im_start|>" in tmpl or arch in ("qwen2", "qwen2moe", "qwen3"):
        return "chatml"
    if "[INST]" in tmpl:
        return "mistral"
    return None


def _read_gguf_md(path: str) -> dict | None:
    try:
        from ..formats.gguf import GGUFReader
        r = GGUFReader(path)
        md = dict(r.metadata)
        md["__n_tensors__"] = len(r.tensors)
        r.close()
        return md
    except Exception as ex:  # not a GGUF (safetensors dir, onnx, ...)
        log.debug("no GGUF metadata for %s: %s", path, ex)
        return None


def guess_defaults(cfg, model_path: str, default_ctx: int = 0):
    if os.environ.get("LOCALAI_DISABLE_GUESSING"):
        return
    if not cfg.parameters.model or not model_path:
        return
    path = os.path.join(model_path, cfg.parameters.model)
    if not os.path.isfile(path):
        return
    md = _read_gguf_md(path)
    if md is None:
        return
    arch = str(md.get("general.architecture", ""))
    ctx_train = md.get(f"{arch}.context_length")
    if cfg.context_size is None:
        cap = default_ctx or int(os.environ.get("LOCALAI_DEFAULT_CONTEXT", "4096"))
        cfg.context_size = int(min(int(ctx_train), cap)) if ctx_train else cap
    if cfg.gpu_layers is None:
        cfg.gpu_layers = 99999999  # everything on the GPU (reference defaultNGPULayers)
    if cfg.has_template() or cfg.template.use_tokenizer_template:
        return
    fam = identify_family(md)
    if fam is None:
        if md.get("tokenizer.chat_template"):
            cfg.template.use_tokenizer_template = True
            cfg.template.jinja_template = True
        return
    spec = FAMILIES[fam]
    for k, v in spec["template"].items():
        setattr(cfg.template, k, v)
    cfg.stopwords = list(dict.fromkeys(list(cfg.stopwords) + spec["stop"]))
    if "repeat_penalty" in spec and not cfg.parameters.repeat_penalty:
        cfg.parameters.repeat_penalty = spec["repeat_penalty"]
    cfg.extra.setdefault("guessed_family", fam)
