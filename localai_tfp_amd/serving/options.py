"""Model config -> gRPC option messages (behavioural parity: core/backend/options.go:
ModelOptions / grpcModelOpts / gRPCPredictOpts)."""
from __future__ import annotations

import os
import random

from ..grpc import pb

RAND_SEED = -1


def _seed(c) -> int:
    s = c.parameters.seed if c.parameters.seed is not None else RAND_SEED
    return random.randint(0, 2**31 - 1) if s == RAND_SEED else int(s)


def model_options(c, app=None, model_path: str = "") -> object:
    d = c.diffusers
    triggers = [pb.GrammarTrigger(word=t.get("word", "") if isinstance(t, dict) else str(t))
                for t in (c.function.grammar.triggers or [])]
    threads = app.threads if app and app.threads else (c.threads or 1)
    mm = c.limit_mm_per_prompt or {}
    return pb.ModelOptions(
        Model=c.parameters.model, ModelFile=os.path.join(model_path, c.parameters.model) if model_path and
        c.parameters.model and not c.parameters.model.startswith(("synthetic:", "/")) else c.parameters.model,
        ModelPath=model_path, CUDA=c.cuda or d.cuda, SchedulerType=d.scheduler_type, GrammarTriggers=triggers,
        PipelineType=d.pipeline_type, CFGScale=c.cfg_scale, LoraAdapter=c.lora_adapter, LoraScale=c.lora_scale,
        LoraAdapters=list(c.lora_adapters), LoraScales=[float(x) for x in c.lora_scales],
        F16Memory=bool(c.f16), LoraBase=c.lora_base, IMG2IMG=d.img2img, CLIPModel=d.clip_model,
        CLIPSubfolder=d.clip_subfolder, Options=[str(o) for o in c.options], CLIPSkip=int(d.clip_skip),
        ControlNet=d.control_net, ContextSize=int(c.context_size or (app.context_size if app and app.context_size
                                                                     else 4096)),
        Seed=_seed(c), NBatch=int(c.parameters.batch or 0), NoMulMatQ=c.no_mulmatq, DraftModel=c.draft_model,
        AudioPath="", Quantization=c.quantization, LoadFormat=c.load_format,
        GPUMemoryUtilization=c.gpu_memory_utilization, TrustRemoteCode=c.trust_remote_code,
        EnforceEager=c.enforce_eager, SwapSpace=c.swap_space, MaxModelLen=c.max_model_len,
        TensorParallelSize=c.tensor_parallel_size, DisableLogStatus=c.disable_log_stats, DType=c.dtype,
        LimitImagePerPrompt=int(mm.get("image", 0)), LimitVideoPerPrompt=int(mm.get("video", 0)),
        LimitAudioPerPrompt=int(mm.get("audio", 0)), MMProj=c.mmproj, FlashAttention=c.flash_attention,
        CacheTypeKey=c.cache_type_k, CacheTypeValue=c.cache_type_v, NoKVOffload=c.no_kv_offloading,
        YarnExtFactor=c.yarn_ext_factor, YarnAttnFactor=c.yarn_attn_factor, YarnBetaFast=c.yarn_beta_fast,
        YarnBetaSlow=c.yarn_beta_slow, NGQA=c.ngqa, RMSNormEps=c.rms_norm_eps, MLock=bool(c.mmlock),
        RopeFreqBase=c.parameters.rope_freq_base, RopeScaling=c.rope_scaling, Type=c.type,
        RopeFreqScale=c.parameters.rope_freq_scale, NUMA=c.numa, Embeddings=bool(c.embeddings),
        LowVRAM=bool(c.low_vram), NGPULayers=int(c.gpu_layers if c.gpu_layers is not None else 9999999),
        MMap=bool(c.mmap), MainGPU=c.main_gpu, Threads=int(threads), TensorSplit=c.tensor_split,
        Tokenizer=c.parameters.tokenizer,
    )


def predict_options(c, model_path: str = "") -> object:
    p = c.parameters
    cache_path = ""
    if c.prompt_cache_path:
        cache_path = os.path.join(model_path, c.prompt_cache_path)
        os.makedirs(os.path.dirname(cache_path) or ".", exist_ok=True)
    return pb.PredictOptions(
        Temperature=float(p.temperature if p.temperature is not None else 0.9),
        TopP=float(p.top_p if p.top_p is not None else 0.95), NDraft=int(c.n_draft),
        TopK=int(p.top_k if p.top_k is not None else 40),
        Tokens=int(p.max_tokens if p.max_tokens is not None else 0), Threads=int(c.threads or 1),
        PromptCacheAll=c.prompt_cache_all, PromptCacheRO=c.prompt_cache_ro, PromptCachePath=cache_path,
        F16KV=bool(c.f16), DebugMode=bool(c.debug), Grammar=c.grammar, NegativePromptScale=p.negative_prompt_scale,
        RopeFreqBase=p.rope_freq_base, RopeFreqScale=p.rope_freq_scale, NegativePrompt=p.negative_prompt,
        Mirostat=int(c.mirostat or 0), MirostatETA=float(c.mirostat_eta if c.mirostat_eta is not None else 0.1),
        MirostatTAU=float(c.mirostat_tau if c.mirostat_tau is not None else 5.0), Debug=bool(c.debug),
        StopPrompts=[s for s in c.stopwords if s], Repeat=int(p.repeat_last_n),
        FrequencyPenalty=float(p.frequency_penalty), PresencePenalty=float(p.presence_penalty),
        Penalty=float(p.repeat_penalty), NKeep=int(p.n_keep), Batch=int(p.batch), IgnoreEOS=p.ignore_eos,
        Seed=_seed(c), MLock=bool(c.mmlock), MMap=bool(c.mmap), MainGPU=c.main_gpu, TensorSplit=c.tensor_split,
        TailFreeSamplingZ=float(p.tfz if p.tfz is not None else 1.0),
        TypicalP=float(p.typical_p if p.typical_p is not None else 1.0),
    )
