"""CTranslate2 model directories (`model.bin` + `config.json` + vocabulary): the format of the reference's
`faster-whisper` backend (backend/python/faster-whisper/backend.py:26-62 loads
`WhisperModel(model_dir, compute_type=...)`). Read without ctranslate2: the binary is a flat list of named
variables,

    u32 binary version | str spec name | u32 spec revision | u32 n_variables
    n x ( str name | u8 rank | rank x u32 dim | u8 dtype | u32 n_bytes | bytes )
    u32 n_aliases | n x ( str alias | str variable )
    str = u16 length (incl. NUL) | utf-8 bytes | NUL

dtype ids: 0 float32, 1 int8, 2 int16, 3 int32, 4 float16, 5 bfloat16. Quantised (int8) weights carry a
`<name>_scale` variable (per output row): w = q / scale. Scalar spec attributes (e.g. `encoder/num_heads`)
are 0-rank variables. A writer for the same layout serves tests and converters.
"""
from __future__ import annotations

import io
import struct

import numpy as np

_DT = {0: np.float32, 1: np.int8, 2: np.int16, 3: np.int32, 4: np.float16}
_DT_ID = {np.dtype(v): k for k, v in _DT.items()}
BF16 = 5


def _rd_str(f) -> str:
    (n,) = struct.unpack("<H", f.read(2))
    s = f.read(n)
    return s[:-1].decode("utf-8") if s.endswith(b"\0") else s.decode("utf-8")


def read_model_bin(path: str) -> tuple[dict, dict]:
    """-> ({variable name: numpy array (float16 / bfloat16 -> float32)}, {"version", "spec", "revision"})."""
    with open(path, "rb") as fh:
        f = io.BufferedReader(fh)
        (version,) = struct.unpack("<I", f.read(4))
        if version < 3 or version > 8:
            raise ValueError(f"{path}: unsupported CTranslate2 binary version {version}")
        spec = _rd_str(f)
        (revision,) = struct.unpack("<I", f.read(4))
        (n,) = struct.unpack("<I", f.read(4))
        out = {}
        for _ in range(n):
            name = _rd_str(f)
            (rank,) = struct.unpack("<B", f.read(1))
            shape = struct.unpack(f"<{rank}I", f.read(4 * rank)) if rank else ()
            (dt,) = struct.unpack("<B", f.read(1))
            (nb,) = struct.unpack("<I", f.read(4))
            raw = f.read(nb)
            if dt == BF16:
                a = (np.frombuffer(raw, np.uint16).astype(np.uint32) << 16).view(np.float32)
            elif dt in _DT:
                a = np.frombuffer(raw, _DT[dt])
            else:
                raise ValueError(f"{path}: variable {name!r} has unknown dtype id {dt}")
            out[name] = a.reshape(shape).copy()
        tail = f.read(4)
        if len(tail) == 4:
            (na,) = struct.unpack("<I", tail)
            for _ in range(na):
                alias, target = _rd_str(f), _rd_str(f)
                if target in out:
                    out[alias] = out[target]
    return out, {"version": version, "spec": spec, "revision": revision}


def write_model_bin(path: str, variables: dict, spec: str, revision: int = 1, version: int = 6,
                    aliases: dict | None = None):
    def w_str(f, s):
        b = s.encode("utf-8")
        f.write(struct.pack("<H", len(b) + 1) + b + b"\0")
    with open(path, "wb") as f:
        f.write(struct.pack("<I", version))
        w_str(f, spec)
        f.write(struct.pack("<I", revision))
        f.write(struct.pack("<I", len(variables)))
        for name, a in variables.items():
            a = np.asarray(a)
            a = a if a.flags.c_contiguous else a.copy()  # keep 0-rank scalars 0-rank
            w_str(f, name)
            f.write(struct.pack("<B", a.ndim))
            for d in a.shape:
                f.write(struct.pack("<I", d))
            f.write(struct.pack("<B", _DT_ID[a.dtype]))
            raw = a.astype(a.dtype.newbyteorder("<")).tobytes()
            f.write(struct.pack("<I", len(raw)))
            f.write(raw)
        aliases = aliases or {}
        f.write(struct.pack("<I", len(aliases)))
        for k, v in aliases.items():
            w_str(f, k)
            w_str(f, v)


def dequantize_vars(v: dict) -> dict:
    """int8 weights with `<name>_scale` -> float32 (w = q / scale); float16 -> float32; scales dropped."""
    out = {}
    for k, a in v.items():
        if k.endswith("_scale") and k[:-6] in v:
            continue
        s = v.get(k + "_scale")
        if s is not None and a.dtype == np.int8:
            a = a.astype(np.float32) / np.asarray(s, np.float32).reshape((-1,) + (1,) * (a.ndim - 1))
        elif a.dtype in (np.float16,):
            a = a.astype(np.float32)
        out[k] = a
    return out


# ---- Whisper (WhisperSpec) -> OpenAI / whisper.cpp tensor names ----------------------------------
def whisper_to_openai(v: dict) -> tuple[dict, dict]:
    """CTranslate2 WhisperSpec variables -> ({OpenAI name: float32}, {"enc_heads", "dec_heads"})."""
    v = dequantize_vars(v)
    out = {}
    d_a = int(v["encoder/conv1/weight"].shape[0])
    d_t = int(v["decoder/embeddings/weight"].shape[1])

    def put(name, a):
        out[name] = np.asarray(a, np.float32)

    put("encoder.conv1.weight", v["encoder/conv1/weight"])
    put("encoder.conv1.bias", v["encoder/conv1/bias"])
    put("encoder.conv2.weight", v["encoder/conv2/weight"])
    put("encoder.conv2.bias", v["encoder/conv2/bias"])
    put("encoder.positional_embedding", v["encoder/position_encodings/encodings"])
    put("encoder.ln_post.weight", v["encoder/layer_norm/gamma"])
    put("encoder.ln_post.bias", v["encoder/layer_norm/beta"])
    put("decoder.token_embedding.weight", v["decoder/embeddings/weight"])
    put("decoder.positional_embedding", v["decoder/position_encodings/encodings"])
    put("decoder.ln.weight", v["decoder/layer_norm/gamma"])
    put("decoder.ln.bias", v["decoder/layer_norm/beta"])

    def ln(src, dst):
        put(dst + ".weight", v[src + "/gamma"])
        put(dst + ".bias", v[src + "/beta"])

    def fused(src, dst, names, d):
        w, b = v[src + "/weight"], v.get(src + "/bias")
        for j, nm in enumerate(names):
            put(f"{dst}.{nm}.weight", w[j * d:(j + 1) * d])
            if b is not None and nm != "key":  # Whisper's key projections have no bias (CT2 stores zeros)
                put(f"{dst}.{nm}.bias", b[j * d:(j + 1) * d])

    def lin(src, dst):
        put(dst + ".weight", v[src + "/weight"])
        if src + "/bias" in v:
            put(dst + ".bias", v[src + "/bias"])

    for side, d in (("encoder", d_a), ("decoder", d_t)):
        i = 0
        while f"{side}/layer_{i}/self_attention/linear_0/weight" in v:
            p, q = f"{side}/layer_{i}", f"{side}.blocks.{i}"
            ln(f"{p}/self_attention/layer_norm", f"{q}.attn_ln")
            fused(f"{p}/self_attention/linear_0", f"{q}.attn", ("query", "key", "value"), d)
            lin(f"{p}/self_attention/linear_1", f"{q}.attn.out")
            if side == "decoder":
                ln(f"{p}/attention/layer_norm", f"{q}.cross_attn_ln")
                lin(f"{p}/attention/linear_0", f"{q}.cross_attn.query")
                fused(f"{p}/attention/linear_1", f"{q}.cross_attn", ("key", "value"), d)
                lin(f"{p}/attention/linear_2", f"{q}.cross_attn.out")
            ln(f"{p}/ffn/layer_norm", f"{q}.mlp_ln")
            lin(f"{p}/ffn/linear_0", f"{q}.mlp.0")
            lin(f"{p}/ffn/linear_1", f"{q}.mlp.2")
            i += 1
    heads = {"enc_heads": int(np.asarray(v.get("encoder/num_heads", d_a // 64)).reshape(-1)[0]),
             "dec_heads": int(np.asarray(v.get("decoder/num_heads", d_t // 64)).reshape(-1)[0])}
    return out, heads
