"""Cooperative bidirectional LSTM (audio.hip lstm_bidir_coop, ops/rnn.py) against torch.nn.LSTM in fp32 (the
Kokoro / StyleTTS 2 shapes: H = 256, input 512 / 640; and H = 128)."""
import pytest
import torch

DEV = "cuda"


def _params(C, H, seed):
    g = torch.Generator().manual_seed(seed)
    p = {}
    for sfx in ("", "_reverse"):
        p[f"l.weight_ih_l0{sfx}"] = torch.randn(4 * H, C, generator=g) * 0.08
        p[f"l.weight_hh_l0{sfx}"] = torch.randn(4 * H, H, generator=g) * 0.08
        p[f"l.bias_ih_l0{sfx}"] = torch.randn(4 * H, generator=g) * 0.1
        p[f"l.bias_hh_l0{sfx}"] = torch.randn(4 * H, generator=g) * 0.1
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("C,H,T", [(512, 256, 37), (640, 256, 160), (96, 128, 1), (256, 128, 64)])
def test_lstm_bidir_matches_torch(C, H, T):
    from localai_tfp_amd.ops.rnn import _ref, lstm_bidir
    p = _params(C, H, C + T)
    x = torch.randn(T, C, generator=torch.Generator().manual_seed(T))
    ref = _ref(x, p, "l")
    pd = {k: v.to(DEV) for k, v in p.items()}
    cache = {}
    got = lstm_bidir(x.to(DEV), pd, "l", cache)
    got2 = lstm_bidir(x.to(DEV), pd, "l", cache)  # cached weights, counters re-zeroed per call
    torch.cuda.synchronize()
    assert got.shape == (T, 2 * H)
    err = float((got.cpu() - ref).abs().max())
    assert err < 2e-4, err
    assert torch.equal(got, got2)


@pytest.mark.gpu
@pytest.mark.parametrize("H,L,T,B", [(512, 2, 45, 1), (256, 1, 9, 2), (128, 2, 1, 1), (1024, 2, 33, 1)])
def test_lstm_stack_matches_torch(H, L, T, B):
    """Unidirectional multi-layer LSTM on the cooperative scan (EnCodec's decoder SLSTM: H = 512, 2 layers)."""
    from localai_tfp_amd.ops.rnn import LSTMStack
    torch.manual_seed(H + T)
    m = torch.nn.LSTM(H, H, L)
    with torch.no_grad():
        for prm in m.parameters():
            prm.mul_(0.6)
    x = torch.randn(T, B, H)
    ref = m(x)[0]
    st = LSTMStack(m.to(DEV))
    got = st(x.to(DEV))
    torch.cuda.synchronize()
    assert got.shape == (T, B, H)
    err = float((got.cpu() - ref).abs().max())
    assert err < 3e-4, err
