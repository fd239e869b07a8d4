"""Compel-style prompt weighting (reference: COMPEL=1 in backend/python/diffusers/backend.py:40-46,230-236):
the syntax parser and its application to the SD1 / SDXL CLIP conditioning. Compel itself is not available,
so parity with its exact embeddings is unpinned; the tests pin the definition (weight 1 == plain prompt,
empty + w * (prompt - empty) per weighted token)."""
import pytest
import torch

from localai_tfp_amd.models.diffusion import prompt_weights as PW
from localai_tfp_amd.models.diffusion.sd_pipeline import UNetPipeline


def test_parse_syntax():
    assert PW.parse("a cat") == [("a cat", 1.0)]
    c = PW.parse("a (red car)1.3 on a road")
    assert c[1] == ("red car", 1.3)
    c = dict(PW.parse("a red car++ in the rain--"))
    assert c["car"] == pytest.approx(1.21) and c["rain"] == pytest.approx(0.81)
    c = dict(PW.parse("(a (big)++ dog)0.5"))
    assert c["big"] == pytest.approx(0.5 * 1.21)
    assert dict(PW.parse("(masterpiece:1.2), cat"))["masterpiece"] == pytest.approx(1.2)
    assert PW.parse("x (unbalanced") == [("x unbalanced", 1.0)]
    assert not PW.has_weights("well-known art") and PW.has_weights("(art)")


@pytest.mark.parametrize("name", ["sd15-test", "sdxl-test"])
def test_weighted_conditioning(name, monkeypatch):
    p = UNetPipeline.synthetic(name, "cpu")
    monkeypatch.setenv("COMPEL", "1")
    plain, pooled = p.encode_prompts(["a red car"])
    same, pooled2 = p.encode_prompts(["(a red car)1.0"])
    assert torch.allclose(same, plain, atol=1e-5)  # weight 1 (syntax only) == the plain prompt
    w, _ = p.encode_prompts(["a (red)1.5 car"])
    empty, _ = p.encode_prompts([""])
    ids, ws = PW.weighted_ids(p.tok1, "a (red)1.5 car")
    k = ws.index(1.5)
    assert torch.allclose(w[0, k] - empty[0, k], 1.5 * (plain[0, k] - empty[0, k]), atol=1e-4)
    assert torch.allclose(w[0, :k], plain[0, :k], atol=1e-5)
    monkeypatch.setenv("COMPEL", "0")
    off, _ = p.encode_prompts(["a (red)1.5 car"])  # off: the syntax is plain text, as without Compel
    assert not torch.allclose(off, w)
