"""Per-model YAML configuration (schema-compatible with the reference's BackendConfig,
core/config/backend_config.go:27-207, so existing gallery / models-dir YAML files load unchanged).

Fields are declared once as dataclasses; `from_dict` maps YAML keys (snake_case as in the
reference's yaml tags) onto them, keeps unknown keys in `extra`, and `to_dict` round-trips.
Defaults and validation follow SetDefaults/Validate (backend_config.go:287-424).
"""
from __future__ import annotations

import dataclasses
import os
import random
import re
import typing
from dataclasses import dataclass, field

RAND_SEED = -1


def _from(cls, d):
    """Recursive dataclass construction from a (YAML) dict; unknown keys land in `extra`."""
    if d is None:
        return cls()
    if isinstance(d, cls):
        return d
    hints = typing.get_type_hints(cls)
    kw = {}
    extra = {}
    names = {f.metadata.get("yaml", f.name): f for f in dataclasses.fields(cls)}
    for k, v in d.items():
        f = names.get(k)
        if f is None or f.metadata.get("skip"):
            extra[k] = v
            continue
        t = hints[f.name]
        origin = typing.get_origin(t)
        args = typing.get_args(t)
        inner = t
        if origin is typing.Union:
            inner = next((a for a in args if a is not type(None)), t)
        if dataclasses.is_dataclass(inner) and isinstance(v, dict):
            v = _from(inner, v)
        kw[f.name] = v
    obj = cls(**kw)
    if hasattr(obj, "extra"):
        obj.extra.update(extra)
    return obj


def _to(obj):
    out = {}
    for f in dataclasses.fields(obj):
        if f.metadata.get("skip") or f.name == "extra":
            continue
        v = getattr(obj, f.name)
        if v is None or v == "" or v == [] or v == {}:
            continue
        if dataclasses.is_dataclass(v):
            v = _to(v)
            if not v:
                continue
        out[f.metadata.get("yaml", f.name)] = v
    if getattr(obj, "extra", None):
        out.update(obj.extra)
    return out


def Y(name, default=None, **kw):
    """Field with an explicit YAML key; `default` may be a factory (list, dict, a dataclass)."""
    if default in (list, dict) or dataclasses.is_dataclass(default):
        return field(default_factory=default, metadata={"yaml": name, **kw})
    return field(default=default, metadata={"yaml": name, **kw})


@dataclass
class PredictionOptions:
    """`parameters:` block (core/schema/prediction.go:3-50)."""
    model: str = ""
    language: str = ""
    translate: bool = False
    n: int = 0
    top_p: float | None = None
    top_k: int | None = None
    temperature: float | None = None
    max_tokens: int | None = Y("max_tokens")
    echo: bool = False
    batch: int = 0
    ignore_eos: bool = False
    repeat_penalty: float = 0.0
    repeat_last_n: int = 0
    n_keep: int = 0
    frequency_penalty: float = 0.0
    presence_penalty: float = 0.0
    tfz: float | None = None
    typical_p: float | None = None
    seed: int | None = None
    negative_prompt: str = ""
    rope_freq_base: float = 0.0
    rope_freq_scale: float = 0.0
    negative_prompt_scale: float = 0.0
    clip_skip: int = 0
    tokenizer: str = ""
    extra: dict = Y("__extra__", dict, skip=True)


@dataclass
class TemplateConfig:
    chat: str = ""
    chat_message: str = ""
    completion: str = ""
    edit: str = ""
    function: str = ""
    use_tokenizer_template: bool = False
    join_chat_messages_by_character: str | None = None
    multimodal: str = ""
    jinja_template: bool = False
    reply_prefix: str = ""
    extra: dict = Y("__extra__", dict, skip=True)


@dataclass
class GrammarConfig:
    parallel_calls: bool = False
    disable_parallel_new_lines: bool = False
    mixed_mode: bool = False
    no_mixed_free_string: bool = False
    no_grammar: bool = False
    prefix: str = ""
    expect_strings_after_json: bool = False
    properties_order: str = ""
    schema_type: str = ""
    triggers: list = Y("triggers", list)
    extra: dict = Y("__extra__", dict, skip=True)


@dataclass
class FunctionsConfig:
    """`function:` block (pkg/functions/parse.go:62-120)."""
    disable_no_action: bool = False
    grammar: GrammarConfig = Y("grammar", GrammarConfig)
    no_action_function_name: str = ""
    no_action_description_name: str = ""
    response_regex: list = Y("response_regex", list)
    json_regex_match: list = Y("json_regex_match", list)
    argument_regex: list = Y("argument_regex", list)
    argument_regex_key_name: str = ""
    argument_regex_value_name: str = ""
    replace_function_results: list = Y("replace_function_results", list)
    replace_llm_results: list = Y("replace_llm_results", list)
    capture_llm_results: list = Y("capture_llm_results", list)
    function_name_key: str = ""
    function_arguments_key: str = ""
    extra: dict = Y("__extra__", dict, skip=True)


@dataclass
class DiffusersConfig:
    cuda: bool = False
    pipeline_type: str = ""
    scheduler_type: str = ""
    enable_parameters: str = ""
    img2img: bool = False
    clip_skip: int = 0
    clip_model: str = ""
    clip_subfolder: str = ""
    control_net: str = ""
    extra: dict = Y("__extra__", dict, skip=True)


@dataclass
class GRPCConfig:
    attempts: int = 0
    attempts_sleep_time: int = 0
    extra: dict = Y("__extra__", dict, skip=True)


@dataclass
class TTSConfig:
    voice: str = ""
    audio_path: str = ""
    extra: dict = Y("__extra__", dict, skip=True)


# use-case flags (backend_config.go:432-449)
FLAG_ANY, FLAG_CHAT, FLAG_COMPLETION, FLAG_EDIT = 0, 1, 2, 4
FLAG_EMBEDDINGS, FLAG_RERANK, FLAG_IMAGE, FLAG_TRANSCRIPT = 8, 16, 32, 64
FLAG_TTS, FLAG_SOUND_GENERATION, FLAG_TOKENIZE, FLAG_VAD, FLAG_VIDEO = 128, 256, 512, 1024, 2048
FLAG_LLM = FLAG_CHAT | FLAG_COMPLETION | FLAG_EDIT
USECASE_FLAGS = {
    "FLAG_ANY": FLAG_ANY, "FLAG_CHAT": FLAG_CHAT, "FLAG_COMPLETION": FLAG_COMPLETION, "FLAG_EDIT": FLAG_EDIT,
    "FLAG_EMBEDDINGS": FLAG_EMBEDDINGS, "FLAG_RERANK": FLAG_RERANK, "FLAG_IMAGE": FLAG_IMAGE,
    "FLAG_TRANSCRIPT": FLAG_TRANSCRIPT, "FLAG_TTS": FLAG_TTS, "FLAG_SOUND_GENERATION": FLAG_SOUND_GENERATION,
    "FLAG_TOKENIZE": FLAG_TOKENIZE, "FLAG_VAD": FLAG_VAD, "FLAG_LLM": FLAG_LLM, "FLAG_VIDEO": FLAG_VIDEO,
}

IMAGE_BACKENDS = ("diffusers", "stablediffusion", "stablediffusion-ggml", "mx-sd")
TTS_BACKENDS = ("bark-cpp", "parler-tts", "piper", "transformers-musicgen", "mx-tts", "kokoro", "coqui", "bark")
LLM_TOKENIZE_BACKENDS = ("llama-cpp", "llama.cpp", "llama", "mx-llm", "rwkv", "")


@dataclass
class ModelConfig:
    name: str = ""
    parameters: PredictionOptions = Y("parameters", PredictionOptions)
    f16: bool | None = None
    threads: int | None = None
    debug: bool | None = None
    roles: dict = Y("roles", dict)
    embeddings: bool | None = None
    backend: str = ""
    template: TemplateConfig = Y("template", TemplateConfig)
    known_usecases: list = Y("known_usecases", list)
    function: FunctionsConfig = Y("function", FunctionsConfig)
    feature_flags: dict = Y("feature_flags", dict)
    # LLMConfig (inline)
    system_prompt: str = ""
    tensor_split: str = ""
    main_gpu: str = ""
    rms_norm_eps: float = 0.0
    ngqa: int = 0
    prompt_cache_path: str = ""
    prompt_cache_all: bool = False
    prompt_cache_ro: bool = False
    mirostat_eta: float | None = None
    mirostat_tau: float | None = None
    mirostat: int | None = None
    gpu_layers: int | None = None
    mmap: bool | None = None
    mmlock: bool | None = None
    low_vram: bool | None = None
    grammar: str = ""
    stopwords: list = Y("stopwords", list)
    cutstrings: list = Y("cutstrings", list)
    extract_regex: list = Y("extract_regex", list)
    trimspace: list = Y("trimspace", list)
    trimsuffix: list = Y("trimsuffix", list)
    context_size: int | None = None
    numa: bool = False
    lora_adapter: str = ""
    lora_base: str = ""
    lora_adapters: list = Y("lora_adapters", list)
    lora_scales: list = Y("lora_scales", list)
    lora_scale: float = 0.0
    no_mulmatq: bool = False
    draft_model: str = ""
    n_draft: int = 0
    quantization: str = ""
    load_format: str = ""
    gpu_memory_utilization: float = 0.0
    trust_remote_code: bool = False
    enforce_eager: bool = False
    swap_space: int = 0
    max_model_len: int = 0
    tensor_parallel_size: int = 0
    disable_log_stats: bool = False
    dtype: str = ""
    limit_mm_per_prompt: dict = Y("limit_mm_per_prompt", dict)
    mmproj: str = ""
    flash_attention: bool = False
    no_kv_offloading: bool = False
    cache_type_k: str = ""
    cache_type_v: str = ""
    rope_scaling: str = ""
    type: str = ""
    yarn_ext_factor: float = 0.0
    yarn_attn_factor: float = 0.0
    yarn_beta_fast: float = 0.0
    yarn_beta_slow: float = 0.0
    cfg_scale: float = 0.0
    # diffusers / misc
    diffusers: DiffusersConfig = Y("diffusers", DiffusersConfig)
    step: int = 0
    grpc: GRPCConfig = Y("grpc", GRPCConfig)
    tts: TTSConfig = Y("tts", TTSConfig)
    cuda: bool = False
    download_files: list = Y("download_files", list)
    description: str = ""
    usage: str = ""
    options: list = Y("options", list)
    # this framework's extensions (ignored by the reference)
    data_parallel: int = 0
    extra: dict = Y("__extra__", dict, skip=True)
    # request-scoped, never serialised
    prompt_strings: list = Y("-prompt_strings", list, skip=True)
    input_strings: list = Y("-input_strings", list, skip=True)
    input_tokens: list = Y("-input_tokens", list, skip=True)
    function_call_string: str = Y("-fcs", "", skip=True)
    function_call_name: str = Y("-fcn", "", skip=True)
    response_format: str = Y("-rf", "", skip=True)
    response_format_map: dict | None = Y("-rfm", None, skip=True)
    source_file: str = Y("-src", "", skip=True)

    # ------------------------------------------------------------------ (de)serialisation
    @classmethod
    def from_dict(cls, d: dict) -> "ModelConfig":
        d = dict(d or {})
        c = _from(cls, d)
        return c

    def to_dict(self) -> dict:
        return _to(self)

    @property
    def model(self) -> str:
        return self.parameters.model

    # ------------------------------------------------------------------ defaults / validation
    def set_defaults(self, ctx_size: int = 0, threads: int = 0, f16: bool = False, debug: bool = False,
                     model_path: str = ""):
        p = self.parameters
        if p.seed is None:
            p.seed = RAND_SEED
        if p.top_k is None:
            p.top_k = 40
        if p.typical_p is None:
            p.typical_p = 1.0
        if p.tfz is None:
            p.tfz = 1.0
        if self.mmap is None:
            self.mmap = os.environ.get("XPU", "") == ""
        if self.mmlock is None:
            self.mmlock = False
        if p.top_p is None:
            p.top_p = 0.95
        if p.temperature is None:
            p.temperature = 0.9
        if p.max_tokens is None:
            p.max_tokens = 0
        if self.mirostat is None:
            self.mirostat = 0
        if self.mirostat_eta is None:
            self.mirostat_eta = 0.1
        if self.mirostat_tau is None:
            self.mirostat_tau = 5.0
        if self.low_vram is None:
            self.low_vram = False
        if self.embeddings is None:
            self.embeddings = False
        if self.threads is None:
            self.threads = threads or 4
        if self.f16 is None:
            self.f16 = f16
        if self.debug is None:
            self.debug = debug
        if debug:
            self.debug = True
        from .guesser import guess_defaults
        guess_defaults(self, model_path, ctx_size)

    def validate(self) -> bool:
        targets = [self.backend, self.parameters.model, self.mmproj] + [
            (f.get("filename", "") if isinstance(f, dict) else "") for f in self.download_files]
        for n in targets:
            if not n:
                continue
            if n.startswith(os.sep) or ".." in n:
                return False
        if self.backend:
            return re.fullmatch(r"[a-zA-Z0-9\-_.]+", self.backend) is not None
        return True

    def has_template(self) -> bool:
        t = self.template
        return bool(t.completion or t.edit or t.chat or t.chat_message)

    # ------------------------------------------------------------------ use cases
    def usecase_flags(self) -> int | None:
        if not self.known_usecases:
            return None
        r = FLAG_ANY
        for s in self.known_usecases:
            r |= USECASE_FLAGS.get("FLAG_" + str(s).upper(), 0)
        return r

    def has_usecases(self, u: int) -> bool:
        k = self.usecase_flags()
        if k is not None and (u & k) == u:
            return True
        return self.guess_usecases(u)

    def guess_usecases(self, u: int) -> bool:
        t = self.template
        if u & FLAG_CHAT and not (t.chat or t.chat_message or t.use_tokenizer_template or t.jinja_template):
            return False
        if u & FLAG_COMPLETION and not t.completion:
            return False
        if u & FLAG_EDIT and not t.edit:
            return False
        if u & FLAG_EMBEDDINGS and not self.embeddings:
            return False
        if u & FLAG_IMAGE:
            if self.backend not in IMAGE_BACKENDS:
                return False
            if self.backend == "diffusers" and not self.diffusers.pipeline_type:
                return False
        if u & FLAG_VIDEO:
            if self.backend not in ("diffusers", "stablediffusion", "mx-sd"):
                return False
        if u & FLAG_RERANK and self.backend not in ("rerankers", "mx-rerank"):
            return False
        if u & FLAG_TRANSCRIPT and self.backend not in ("whisper", "mx-whisper", "faster-whisper"):
            return False
        if u & FLAG_TTS and self.backend not in TTS_BACKENDS:
            return False
        if u & FLAG_SOUND_GENERATION and self.backend not in ("transformers-musicgen", "mx-tts"):
            return False
        if u & FLAG_TOKENIZE and self.backend not in LLM_TOKENIZE_BACKENDS:
            return False
        if u & FLAG_VAD and self.backend not in ("silero-vad", "mx-vad"):
            return False
        return True

    # ------------------------------------------------------------------ function calling state
    def should_use_functions(self) -> bool:
        return self.function_call_string != "none" or self.should_call_specific_function()

    def should_call_specific_function(self) -> bool:
        return bool(self.function_call_name)

    def function_to_call(self) -> str:
        if self.function_call_name and self.function_call_name not in ("none", "auto"):
            return self.function_call_name
        return self.function_call_string

    def resolved_seed(self) -> int:
        s = self.parameters.seed
        if s is None or s == RAND_SEED:
            return random.randint(0, 2**31 - 1)
        return int(s)

    def copy(self) -> "ModelConfig":
        import copy
        return copy.deepcopy(self)
