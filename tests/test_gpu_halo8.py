"""First-layer conv (Cin 8, Cout 64, 4x4 s2 p1) + LeakyReLU/ReLU epilogue on the row-halo kernel
(csrc/halo8_bf16.hip) against the LDS-DMA GEMM tile it replaces (STC_HALO8=0) -- STCGAN/networks.py:99,165.
Same K order and MFMA instruction: the outputs must be bit-identical, one and two activated outputs, with and
without bias, at the training size (256^2 -> 128^2), the 480x640 inference size, odd-width inputs and a
channel-offset output view (a concat buffer)."""
import os

import pytest
import torch

from stcgan_amd import _lib as L
from stcgan_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16

CASES = [  # (B, H, W, bias, two outputs, output channel offset)
    (32, 256, 256, False, False, 0),
    (32, 256, 256, True, True, 0),
    (2, 480, 640, False, False, 0),
    (3, 38, 54, True, True, 64),
    (1, 2, 2, True, False, 0),
]


def _run(B, H, W, bias, two, c0, halo, monkeypatch):
    monkeypatch.setenv("STC_HALO8", "1" if halo else "0")
    g = torch.Generator(device=DEV).manual_seed(3)
    x = (torch.randn((B, H, W, 8), device=DEV, generator=g)).to(BF)
    w = (torch.randn((1, 64, 16, 8), device=DEV, generator=g) * 0.1).to(BF)
    b = torch.randn(64, device=DEV, generator=g) if bias else None
    oh, ow = H // 2, W // 2
    y1 = torch.full((B, oh, ow, 64 + c0), 3.0, device=DEV, dtype=BF)
    y2 = torch.full((B, oh, ow, 64 + c0), 3.0, device=DEV, dtype=BF)
    ok = ops.conv_act(L.CONV_S2, B, L.nhwc_view(x), 8, w, 64, L.nhwc_view(y1, c0, oh, ow), 0.2, BF,
                      L.nhwc_view(y2, c0, oh, ow) if two else None, 0.0, bias=b)
    assert ok
    torch.cuda.synchronize()
    return y1, y2


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"B{c[0]}_{c[1]}x{c[2]}_bias{int(c[3])}_two{int(c[4])}_c0{c[5]}")
def test_halo8_bit_identical_to_gemm_tile(case, monkeypatch):
    B, H, W, bias, two, c0 = case
    a1, a2 = _run(B, H, W, bias, two, c0, True, monkeypatch)
    r1, r2 = _run(B, H, W, bias, two, c0, False, monkeypatch)
    assert torch.equal(a1, r1)
    assert torch.equal(a2, r2)
    if c0:
        assert bool((a1[..., :c0] == 3.0).all()), "write outside the output view"
    assert float(a1[..., c0:].float().abs().max()) > 0


def test_halo8_matches_torch_conv(monkeypatch):
    """Against torch's fp32 conv2d of the same bf16 operands (LeakyReLU 0.2): bf16 output rounding only."""
    monkeypatch.setenv("STC_HALO8", "1")
    g = torch.Generator(device=DEV).manual_seed(5)
    B, H, W = 4, 64, 96
    x = torch.randn((B, H, W, 8), device=DEV, generator=g).to(BF)
    wt = (torch.randn((64, 8, 4, 4), device=DEV, generator=g) * 0.1)
    w = wt.to(BF).permute(0, 2, 3, 1).reshape(1, 64, 16, 8).contiguous()  # [n][tap][c]
    b = torch.randn(64, device=DEV, generator=g)
    y = torch.zeros((B, H // 2, W // 2, 64), device=DEV, dtype=BF)
    assert ops.conv_act(L.CONV_S2, B, L.nhwc_view(x), 8, w, 64, L.nhwc_view(y), 0.2, BF, bias=b)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wt.to(BF).float(), b, stride=2, padding=1)
    ref = torch.nn.functional.leaky_relu(ref, 0.2).permute(0, 2, 3, 1)
    err = float((y.float() - ref).abs().max())
    assert err <= 2.0 ** -7 * float(ref.abs().max()) + 1e-3, err
