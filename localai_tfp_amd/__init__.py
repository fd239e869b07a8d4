"""localai_tfp_amd — an MI355X-native (gfx950 / CDNA4) local inference server with LocalAI's
OpenAI-compatible API surface, gRPC backend contract, YAML model configs and gallery.

Layers (see SURVEY.md §1 for the reference's layer map):
  gateway/   HTTP API (OpenAI / LocalAI / ElevenLabs / Jina routes), request middleware
  config/    application + per-model YAML configs, GGUF default guessing
  templates/ prompt templates (Go text/template subset + Jinja)
  functions/ tools -> JSON schema -> GBNF grammars, tool-call parsing
  grpc/      backend.proto contract (runtime-built descriptors), client + server
  workers/   backend processes: LLM (this package's engine), embeddings, whisper, SD, stores, VAD, TTS
  engine/    continuous-batching LLM engine: paged KV, scheduler, sampler, grammar, hipGraph decode
  models/    model graphs on the HIP kernels (llama family, bert, whisper, sd)
  ops/       device ops (HIP kernels in csrc/kernels via _native; fp32 PyTorch references on CPU)
  parallel/  tensor parallel (RCCL over xGMI) and data-parallel replicas
"""
__version__ = "0.1.0"
