"""gRPC backend workers (one process per model instance, one GPU per process).

Registry of backend names -> worker modules, with the reference's aliases
(pkg/model/initializers.go:24-41)."""
WORKERS = {
    "llama-cpp": "localai_tfp_amd.workers.llm",
    "mx-llm": "localai_tfp_amd.workers.llm",
    "vllm": "localai_tfp_amd.workers.llm",
    "transformers": "localai_tfp_amd.workers.llm",
    "exllama2": "localai_tfp_amd.workers.llm",
    "bert-embeddings": "localai_tfp_amd.workers.bert",
    "sentencetransformers": "localai_tfp_amd.workers.bert",
    "rerankers": "localai_tfp_amd.workers.bert",
    "whisper": "localai_tfp_amd.workers.whisper",
    "faster-whisper": "localai_tfp_amd.workers.whisper",
    "stablediffusion-ggml": "localai_tfp_amd.workers.diffusion",
    "diffusers": "localai_tfp_amd.workers.diffusion",
    "local-store": "localai_tfp_amd.workers.store",
    "silero-vad": "localai_tfp_amd.workers.vad",
    "piper": "localai_tfp_amd.workers.tts",
    # model families not implemented here: LoadModel fails with an explicit error (workers/unsupported.py)
    "bark": "localai_tfp_amd.workers.bark",  # models/bark.py
    "bark-cpp": "localai_tfp_amd.workers.bark",
    "coqui": "localai_tfp_amd.workers.tts",
    "kokoro": "localai_tfp_amd.workers.kokoro",
    "transformers-musicgen": "localai_tfp_amd.workers.musicgen",  # models/musicgen.py
    "transformers-tts": "localai_tfp_amd.workers.tts",
    "huggingface": "localai_tfp_amd.workers.huggingface",
    "langchain-huggingface": "localai_tfp_amd.workers.huggingface",
}

ALIASES = {
    "llama": "llama-cpp",
    "llama.cpp": "llama-cpp",
    "go-llama": "llama-cpp",
    "sentencetransformers": "transformers",
    "stablediffusion": "stablediffusion-ggml",
    "tinydream": "stablediffusion-ggml",
    "huggingface-embeddings": "bert-embeddings",
    "whisper-ggml": "whisper",
}

# auto-detection order when a model config names no backend (initializers.go:137-179)
AUTODETECT_ORDER = ["llama-cpp", "bert-embeddings", "whisper", "stablediffusion-ggml", "piper", "silero-vad"]


def resolve(name: str) -> str:
    n = (name or "").strip().lower()
    if n in WORKERS:  # a registered name wins over an alias (sentencetransformers -> the BERT worker)
        return n
    return ALIASES.get(n, n)
