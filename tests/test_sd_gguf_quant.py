"""SD3.5-medium from the gallery's stablediffusion-ggml files (gallery/index.yaml sd-3.5-medium-ggml:
sd3.5_medium-Q4_0.gguf + clip_l/clip_g/t5xxl-Q4_0.gguf; gosd.cpp:56-162): the GGUF block weights of the
MMDiT-X transformer and the three text encoders stay quantised (nn.QParam over ops.linear.QWeight) and
must match the same files loaded dense (dequantised fp32) — on CPU through the reference GEMM, on the
GPU through the quantised MFMA kernels. Files are synthetic (random weights in the exact Stability / HF
tensor layouts, Q4_0 blocks as sd.cpp writes them); parity with stable-diffusion.cpp is unpinned."""
import numpy as np
import pytest
import torch
import yaml

from localai_tfp_amd.models.diffusion import single_file as SF
from localai_tfp_amd.models.diffusion.nn import QParam

from test_sd_single_file import _mmdit_to_sai, _vae_to_ldm


def _save_q4_0(path, sd, arch):
    """2-D matrices with 32-aligned rows as Q4_0 blocks (sd.cpp --type q4_0), everything else fp32."""
    from localai_tfp_amd.formats.gguf import GGUFWriter, QType
    from localai_tfp_amd.ops.quant import quantize_q4_0
    w = GGUFWriter(path)
    w.add("general.architecture", arch)
    for k, v in sd.items():
        a = v.float().numpy()
        if a.ndim == 2 and a.shape[1] % 32 == 0 and "embed" not in k:
            w.add_tensor(k, quantize_q4_0(a).tobytes(), shape=tuple(reversed(a.shape)), qtype=QType.Q4_0)
        else:
            w.add_tensor(k, np.ascontiguousarray(a))
    w.write()


def _write_gallery_files(d):
    from localai_tfp_amd.models.diffusion.pipeline import SD3Pipeline
    ref = SD3Pipeline.synthetic("sd3.5m-qtest", "cpu")
    c = ref.p.mmdit
    msd = _mmdit_to_sai({k: v.contiguous() for k, v in ref.mmdit.state_dict().items()}, c.dim, c.layers)
    f = {"model.diffusion_model." + k: v for k, v in msd.items()}
    f.update({"first_stage_model." + k: v for k, v in _vae_to_ldm(
        {k: v.contiguous() for k, v in ref.vae.state_dict().items()}).items()})
    _save_q4_0(str(d / "sd3.5_medium-Q4_0.gguf"), f, "sd3")
    for name, m in (("clip_l", ref.clip_l), ("clip_g", ref.clip_g), ("t5xxl", ref.t5)):
        _save_q4_0(str(d / f"{name}-Q4_0.gguf"),
                   {f"text_encoders.{name}.transformer.{k}": v.contiguous() for k, v in m.state_dict().items()}, name)
    return ref


OPTS = ["clip_l_path:clip_l-Q4_0.gguf", "clip_g_path:clip_g-Q4_0.gguf", "t5xxl_path:t5xxl-Q4_0.gguf", "sampler:euler"]


def _load(d, device, quant: bool, monkeypatch):
    opts = {o.split(":", 1)[0]: str(d / o.split(":", 1)[1]) for o in OPTS[:3]}
    with monkeypatch.context() as mp:
        if not quant:
            mp.setattr(SF, "_keep_quant", lambda ti: False)
        return SF.from_single_file(str(d / "sd3.5_medium-Q4_0.gguf"), device, opts)


def _nq(m):
    return sum(isinstance(getattr(x, "weight", None), QParam) for x in m.modules())


def _inputs(c):
    g = torch.Generator().manual_seed(0)
    return (torch.randn(2, 16, 16, 16, generator=g), torch.tensor([600.0, 30.0]),
            torch.randn(2, 9, c.joint_dim, generator=g), torch.randn(2, c.pooled_dim, generator=g))


def test_sd35_medium_gguf_stays_quantised_cpu(tmp_path, monkeypatch):
    _write_gallery_files(tmp_path)
    pq = _load(tmp_path, "cpu", True, monkeypatch)
    pd = _load(tmp_path, "cpu", False, monkeypatch)
    c = pq.mmdit.cfg
    assert c.dual_attention_layers == (0, 1) and c.qk_norm
    # every MMDiT linear with a 256-multiple K is quantised (not the 64-wide patch embedding)
    assert _nq(pq.mmdit) >= 40 and _nq(pd.mmdit) == 0
    assert _nq(pq.clip_l) > 0 and _nq(pq.clip_g) > 0 and _nq(pq.t5) > 0
    w = pq.mmdit.transformer_blocks[0].attn2.to_q.weight
    assert isinstance(w, QParam)
    args = _inputs(c)
    with torch.no_grad():
        a, b = pq.mmdit(*args), pd.mmdit(*args)
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-4 * float(b.abs().max()))
        ids = torch.randint(0, 600, (2, 77))
        for x, y in ((pq.clip_l, pd.clip_l), (pq.clip_g, pd.clip_g)):
            ha, pa = x(ids, 599)[:2]
            hb, pb = y(ids, 599)[:2]
            assert torch.allclose(ha, hb, atol=1e-4) and torch.allclose(pa, pb, atol=1e-4)
        tid = torch.randint(0, 300, (2, 16))
        assert torch.allclose(pq.t5(tid), pd.t5(tid), atol=1e-4)


def test_sd35_medium_gallery_yaml_generates(tmp_path):
    """The gallery entry's overrides verbatim (backend stablediffusion-ggml, the three *_path options,
    sampler:euler) load through the model config and the diffusion worker writes a PNG."""
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.diffusion import DiffusionServicer
    _write_gallery_files(tmp_path)
    cfg = {"name": "sd-3.5-medium-ggml", "backend": "stablediffusion-ggml", "options": OPTS,
           "parameters": {"model": "sd3.5_medium-Q4_0.gguf"}}
    (tmp_path / "sd35.yaml").write_text(yaml.safe_dump(cfg))
    s = DiffusionServicer(device="cpu")
    r = s.LoadModel(pb.ModelOptions(Model=cfg["parameters"]["model"], ModelPath=str(tmp_path), Options=OPTS), None)
    assert r.success, r.message
    dst = str(tmp_path / "o.png")
    r = s.GenerateImage(pb.GenerateImageRequest(positive_prompt="a lighthouse", width=32, height=32, step=2, seed=1,
                                                dst=dst), None)
    assert r.success, r.message
    with open(dst, "rb") as f:
        assert f.read(8) == b"\x89PNG\r\n\x1a\n"


@pytest.mark.gpu
def test_sd35_medium_gguf_quantised_gpu(tmp_path, monkeypatch):
    """Quantised weights on the GPU (Q4_0 carried as Q8_0 blocks through the bf16 quantised MFMA GEMM) against
    the dense fp32 CPU path of the same files."""
    _write_gallery_files(tmp_path)
    pg = _load(tmp_path, "cuda", True, monkeypatch)
    pd = _load(tmp_path, "cpu", False, monkeypatch)
    assert _nq(pg.mmdit) >= 40 and _nq(pg.t5) > 0
    args = _inputs(pg.mmdit.cfg)
    with torch.no_grad():
        ref = pd.mmdit(*args)
        got = pg.mmdit(*(a.cuda() for a in args)).float().cpu()
        err = float((got - ref).abs().max() / ref.abs().max())
        assert err < 5e-2, err
        tid = torch.randint(0, 300, (2, 16))
        t_ref, t_got = pd.t5(tid), pg.t5(tid.cuda()).float().cpu()
        assert float((t_got - t_ref).norm() / t_ref.norm()) < 6e-2  # bf16 activations through 2 random layers
        ids = torch.randint(0, 600, (2, 77))
        h_ref = pd.clip_g(ids, 599)[0]
        h_got = pg.clip_g(ids.cuda(), 599)[0].float().cpu()
        assert float((h_got - h_ref).norm() / h_ref.norm()) < 6e-2
    img = pg.generate("a lighthouse", __import__("localai_tfp_amd.models.diffusion.pipeline",
                                                  fromlist=["GenParams"]).GenParams(width=64, height=64, steps=2))
    assert torch.isfinite(img).all()
