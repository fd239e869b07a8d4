"""The backend worker contract (`service backend.Backend`), wire-compatible with the reference's
backend/backend.proto:10-374 (same package, service, method names, message names, field numbers
and types), declared as data and turned into protobuf descriptors at import time.

Why not a .proto + protoc: the image has the protobuf runtime and grpcio but no protoc /
grpcio-tools, so :func:`build_file_descriptor` assembles the ``FileDescriptorProto`` directly and
:func:`render_proto` can emit the equivalent .proto text for other-language clients (e.g. a Go
gateway built elsewhere): ``python -m localai_tfp_amd.grpc.schema > backend.proto``.
"""
from __future__ import annotations

PACKAGE = "backend"
SERVICE = "Backend"

# (name, request, response, server_streaming)
METHODS = [
    ("Health", "HealthMessage", "Reply", False),
    ("Predict", "PredictOptions", "Reply", False),
    ("LoadModel", "ModelOptions", "Result", False),
    ("PredictStream", "PredictOptions", "Reply", True),
    ("Embedding", "PredictOptions", "EmbeddingResult", False),
    ("GenerateImage", "GenerateImageRequest", "Result", False),
    ("GenerateVideo", "GenerateVideoRequest", "Result", False),
    ("AudioTranscription", "TranscriptRequest", "TranscriptResult", False),
    ("TTS", "TTSRequest", "Result", False),
    ("SoundGeneration", "SoundGenerationRequest", "Result", False),
    ("TokenizeString", "PredictOptions", "TokenizationResponse", False),
    ("Status", "HealthMessage", "StatusResponse", False),
    ("StoresSet", "StoresSetOptions", "Result", False),
    ("StoresDelete", "StoresDeleteOptions", "Result", False),
    ("StoresGet", "StoresGetOptions", "StoresGetResult", False),
    ("StoresFind", "StoresFindOptions", "StoresFindResult", False),
    ("Rerank", "RerankRequest", "RerankResult", False),
    ("GetMetrics", "MetricsRequest", "MetricsResponse", False),
    ("VAD", "VADRequest", "VADResponse", False),
]

# field spec: (name, number, type[, label]) ; label in {"", "repeated", "optional"}
# type: scalar name, a message name, or "map<string,uint64>"
F = tuple
MESSAGES: dict[str, list] = {
    "MetricsRequest": [],
    "MetricsResponse": [F(("slot_id", 1, "int32")), F(("prompt_json_for_slot", 2, "string")),
                        F(("tokens_per_second", 3, "float")), F(("tokens_generated", 4, "int32")),
                        F(("prompt_tokens_processed", 5, "int32"))],
    "RerankRequest": [("query", 1, "string"), ("documents", 2, "string", "repeated"), ("top_n", 3, "int32")],
    "RerankResult": [("usage", 1, "Usage"), ("results", 2, "DocumentResult", "repeated")],
    "Usage": [("total_tokens", 1, "int32"), ("prompt_tokens", 2, "int32")],
    "DocumentResult": [("index", 1, "int32"), ("text", 2, "string"), ("relevance_score", 3, "float")],
    "StoresKey": [("Floats", 1, "float", "repeated")],
    "StoresValue": [("Bytes", 1, "bytes")],
    "StoresSetOptions": [("Keys", 1, "StoresKey", "repeated"), ("Values", 2, "StoresValue", "repeated")],
    "StoresDeleteOptions": [("Keys", 1, "StoresKey", "repeated")],
    "StoresGetOptions": [("Keys", 1, "StoresKey", "repeated")],
    "StoresGetResult": [("Keys", 1, "StoresKey", "repeated"), ("Values", 2, "StoresValue", "repeated")],
    "StoresFindOptions": [("Key", 1, "StoresKey"), ("TopK", 2, "int32")],
    "StoresFindResult": [("Keys", 1, "StoresKey", "repeated"), ("Values", 2, "StoresValue", "repeated"),
                         ("Similarities", 3, "float", "repeated")],
    "HealthMessage": [],
    "PredictOptions": [
        ("Prompt", 1, "string"), ("Seed", 2, "int32"), ("Threads", 3, "int32"), ("Tokens", 4, "int32"),
        ("TopK", 5, "int32"), ("Repeat", 6, "int32"), ("Batch", 7, "int32"), ("NKeep", 8, "int32"),
        ("Temperature", 9, "float"), ("Penalty", 10, "float"), ("F16KV", 11, "bool"), ("DebugMode", 12, "bool"),
        ("StopPrompts", 13, "string", "repeated"), ("IgnoreEOS", 14, "bool"), ("TailFreeSamplingZ", 15, "float"),
        ("TypicalP", 16, "float"), ("FrequencyPenalty", 17, "float"), ("PresencePenalty", 18, "float"),
        ("Mirostat", 19, "int32"), ("MirostatETA", 20, "float"), ("MirostatTAU", 21, "float"),
        ("PenalizeNL", 22, "bool"), ("LogitBias", 23, "string"), ("MLock", 25, "bool"), ("MMap", 26, "bool"),
        ("PromptCacheAll", 27, "bool"), ("PromptCacheRO", 28, "bool"), ("Grammar", 29, "string"),
        ("MainGPU", 30, "string"), ("TensorSplit", 31, "string"), ("TopP", 32, "float"),
        ("PromptCachePath", 33, "string"), ("Debug", 34, "bool"), ("EmbeddingTokens", 35, "int32", "repeated"),
        ("Embeddings", 36, "string"), ("RopeFreqBase", 37, "float"), ("RopeFreqScale", 38, "float"),
        ("NegativePromptScale", 39, "float"), ("NegativePrompt", 40, "string"), ("NDraft", 41, "int32"),
        ("Images", 42, "string", "repeated"), ("UseTokenizerTemplate", 43, "bool"),
        ("Messages", 44, "Message", "repeated"), ("Videos", 45, "string", "repeated"),
        ("Audios", 46, "string", "repeated"), ("CorrelationId", 47, "string"),
    ],
    "Reply": [("message", 1, "bytes"), ("tokens", 2, "int32"), ("prompt_tokens", 3, "int32"),
              ("timing_prompt_processing", 4, "double"), ("timing_token_generation", 5, "double")],
    "GrammarTrigger": [("word", 1, "string")],
    "ModelOptions": [
        ("Model", 1, "string"), ("ContextSize", 2, "int32"), ("Seed", 3, "int32"), ("NBatch", 4, "int32"),
        ("F16Memory", 5, "bool"), ("MLock", 6, "bool"), ("MMap", 7, "bool"), ("VocabOnly", 8, "bool"),
        ("LowVRAM", 9, "bool"), ("Embeddings", 10, "bool"), ("NUMA", 11, "bool"), ("NGPULayers", 12, "int32"),
        ("MainGPU", 13, "string"), ("TensorSplit", 14, "string"), ("Threads", 15, "int32"),
        ("LibrarySearchPath", 16, "string"), ("RopeFreqBase", 17, "float"), ("RopeFreqScale", 18, "float"),
        ("RMSNormEps", 19, "float"), ("NGQA", 20, "int32"), ("ModelFile", 21, "string"),
        ("PipelineType", 26, "string"), ("SchedulerType", 27, "string"), ("CUDA", 28, "bool"),
        ("CFGScale", 29, "float"), ("IMG2IMG", 30, "bool"), ("CLIPModel", 31, "string"),
        ("CLIPSubfolder", 32, "string"), ("CLIPSkip", 33, "int32"), ("ControlNet", 48, "string"),
        ("Tokenizer", 34, "string"), ("LoraBase", 35, "string"), ("LoraAdapter", 36, "string"),
        ("LoraScale", 42, "float"), ("NoMulMatQ", 37, "bool"), ("DraftModel", 39, "string"),
        ("AudioPath", 38, "string"), ("Quantization", 40, "string"), ("GPUMemoryUtilization", 50, "float"),
        ("TrustRemoteCode", 51, "bool"), ("EnforceEager", 52, "bool"), ("SwapSpace", 53, "int32"),
        ("MaxModelLen", 54, "int32"), ("TensorParallelSize", 55, "int32"), ("LoadFormat", 58, "string"),
        ("DisableLogStatus", 66, "bool"), ("DType", 67, "string"), ("LimitImagePerPrompt", 68, "int32"),
        ("LimitVideoPerPrompt", 69, "int32"), ("LimitAudioPerPrompt", 70, "int32"), ("MMProj", 41, "string"),
        ("RopeScaling", 43, "string"), ("YarnExtFactor", 44, "float"), ("YarnAttnFactor", 45, "float"),
        ("YarnBetaFast", 46, "float"), ("YarnBetaSlow", 47, "float"), ("Type", 49, "string"),
        ("FlashAttention", 56, "bool"), ("NoKVOffload", 57, "bool"), ("ModelPath", 59, "string"),
        ("LoraAdapters", 60, "string", "repeated"), ("LoraScales", 61, "float", "repeated"),
        ("Options", 62, "string", "repeated"), ("CacheTypeKey", 63, "string"), ("CacheTypeValue", 64, "string"),
        ("GrammarTriggers", 65, "GrammarTrigger", "repeated"),
    ],
    "Result": [("message", 1, "string"), ("success", 2, "bool")],
    "EmbeddingResult": [("embeddings", 1, "float", "repeated")],
    "TranscriptRequest": [("dst", 2, "string"), ("language", 3, "string"), ("threads", 4, "uint32"),
                          ("translate", 5, "bool")],
    "TranscriptResult": [("segments", 1, "TranscriptSegment", "repeated"), ("text", 2, "string")],
    "TranscriptSegment": [("id", 1, "int32"), ("start", 2, "int64"), ("end", 3, "int64"), ("text", 4, "string"),
                          ("tokens", 5, "int32", "repeated")],
    "GenerateImageRequest": [("height", 1, "int32"), ("width", 2, "int32"), ("mode", 3, "int32"),
                             ("step", 4, "int32"), ("seed", 5, "int32"), ("positive_prompt", 6, "string"),
                             ("negative_prompt", 7, "string"), ("dst", 8, "string"), ("src", 9, "string"),
                             ("EnableParameters", 10, "string"), ("CLIPSkip", 11, "int32")],
    "GenerateVideoRequest": [("prompt", 1, "string"), ("start_image", 2, "string"), ("end_image", 3, "string"),
                             ("width", 4, "int32"), ("height", 5, "int32"), ("num_frames", 6, "int32"),
                             ("fps", 7, "int32"), ("seed", 8, "int32"), ("cfg_scale", 9, "float"),
                             ("dst", 10, "string")],
    "TTSRequest": [("text", 1, "string"), ("model", 2, "string"), ("dst", 3, "string"), ("voice", 4, "string"),
                   ("language", 5, "string", "optional")],
    "VADRequest": [("audio", 1, "float", "repeated")],
    "VADSegment": [("start", 1, "float"), ("end", 2, "float")],
    "VADResponse": [("segments", 1, "VADSegment", "repeated")],
    "SoundGenerationRequest": [("text", 1, "string"), ("model", 2, "string"), ("dst", 3, "string"),
                               ("duration", 4, "float", "optional"), ("temperature", 5, "float", "optional"),
                               ("sample", 6, "bool", "optional"), ("src", 7, "string", "optional"),
                               ("src_divisor", 8, "int32", "optional")],
    "TokenizationResponse": [("length", 1, "int32"), ("tokens", 2, "int32", "repeated")],
    "MemoryUsageData": [("total", 1, "uint64"), ("breakdown", 2, "map<string,uint64>")],
    "StatusResponse": [("state", 1, "enum:State"), ("memory", 2, "MemoryUsageData")],
    "Message": [("role", 1, "string"), ("content", 2, "string")],
}

ENUMS = {"StatusResponse.State": [("UNINITIALIZED", 0), ("BUSY", 1), ("READY", 2), ("ERROR", -1)]}

_SCALARS = {
    "double": 1, "float": 2, "int64": 3, "uint64": 4, "int32": 5, "bool": 8, "string": 9, "bytes": 12,
    "uint32": 13,
}
TYPE_MESSAGE, TYPE_ENUM = 11, 14
LABEL_OPTIONAL, LABEL_REPEATED = 1, 3


def build_file_descriptor():
    from google.protobuf import descriptor_pb2 as d
    fd = d.FileDescriptorProto(name="localai_backend.proto", package=PACKAGE, syntax="proto3")
    for mname, fields in MESSAGES.items():
        m = fd.message_type.add(name=mname)
        n_oneof = 0
        for spec in fields:
            name, num, typ = spec[0], spec[1], spec[2]
            label = spec[3] if len(spec) > 3 else ""
            f = m.field.add(name=name, number=num, json_name=name)
            f.label = LABEL_REPEATED if label == "repeated" else LABEL_OPTIONAL
            if typ.startswith("map<"):
                kt, vt = typ[4:-1].split(",")
                entry = m.nested_type.add(name=name[0].upper() + name[1:] + "Entry")
                entry.options.map_entry = True
                entry.field.add(name="key", number=1, type=_SCALARS[kt], label=LABEL_OPTIONAL, json_name="key")
                entry.field.add(name="value", number=2, type=_SCALARS[vt], label=LABEL_OPTIONAL, json_name="value")
                f.type = TYPE_MESSAGE
                f.type_name = f".{PACKAGE}.{mname}.{entry.name}"
                f.label = LABEL_REPEATED
            elif typ.startswith("enum:"):
                ename = typ[5:]
                e = m.enum_type.add(name=ename)
                for vn, vv in ENUMS[f"{mname}.{ename}"]:
                    e.value.add(name=vn, number=vv)
                f.type = TYPE_ENUM
                f.type_name = f".{PACKAGE}.{mname}.{ename}"
            elif typ in _SCALARS:
                f.type = _SCALARS[typ]
            else:
                f.type = TYPE_MESSAGE
                f.type_name = f".{PACKAGE}.{typ}"
            if label == "optional":
                m.oneof_decl.add(name=f"_{name}")
                f.oneof_index = n_oneof
                f.proto3_optional = True
                n_oneof += 1
    svc = fd.service.add(name=SERVICE)
    for name, req, resp, stream in METHODS:
        svc.method.add(name=name, input_type=f".{PACKAGE}.{req}", output_type=f".{PACKAGE}.{resp}",
                       server_streaming=stream)
    return fd


def render_proto() -> str:
    lines = ['syntax = "proto3";', "", f"package {PACKAGE};", "", f"service {SERVICE} {{"]
    for name, req, resp, stream in METHODS:
        lines.append(f"  rpc {name}({req}) returns ({'stream ' if stream else ''}{resp}) {{}}")
    lines.append("}")
    for mname, fields in MESSAGES.items():
        lines += ["", f"message {mname} {{"]
        for spec in fields:
            name, num, typ = spec[0], spec[1], spec[2]
            label = spec[3] + " " if len(spec) > 3 else ""
            if typ.startswith("enum:"):
                en = typ[5:]
                lines.append(f"  enum {en} {{")
                for vn, vv in ENUMS[f"{mname}.{en}"]:
                    lines.append(f"    {vn} = {vv};")
                lines.append("  }")
                typ = en
            lines.append(f"  {label}{typ} {name} = {num};")
        lines.append("}")
    return "\n".join(lines) + "\n"


if __name__ == "__main__":
    print(render_proto())
