"""stc_adam_pack_step: the fused Adam + operand repack against torch.optim.Adam (the update) and
stc_pack_weight of the updated weight (every packed layout, bit-exact), incl. ragged 16x16 tiles."""
import pytest
import torch

from stcgan_amd import _lib as L
from stcgan_amd import ops
from stcgan_amd.optim import Adam

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _gen(shape, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g)


@pytest.mark.parametrize("P,Q,modes,dt", [
    (64, 3, (L.PACK_CONV_FWD, L.PACK_CONV_DGRAD), torch.bfloat16),
    (40, 24, (L.PACK_CONVT_FWD, L.PACK_CONVT_DGRAD), torch.bfloat16),
    (17, 33, (L.PACK_CONV_FWD, L.PACK_CONV_S1_DGRAD), torch.bfloat16),
    (32, 16, (L.PACK_CONV_FWD, L.PACK_CONV_DGRAD, L.PACK_CONV_S1_DGRAD), torch.bfloat16),
    (24, 40, (L.PACK_CONVT_FWD, L.PACK_CONVT_DGRAD), torch.float32),
])
def test_adam_pack_matches_adam_then_pack(P, Q, modes, dt):
    w = torch.nn.Parameter(_gen((P, Q, 4, 4), P * Q).to(DEV))
    b = torch.nn.Parameter(_gen((P,), 7).to(DEV))
    ref_w = torch.nn.Parameter(w.detach().cpu().clone())
    ref_b = torch.nn.Parameter(b.detach().cpu().clone())
    opt = Adam([w, b], lr=5e-5, betas=(0.5, 0.999))
    ropt = torch.optim.Adam([ref_w, ref_b], lr=5e-5, betas=(0.5, 0.999))
    cache = {}
    pads = {m: ((Q if m in (L.PACK_CONV_DGRAD, L.PACK_CONV_S1_DGRAD, L.PACK_CONVT_FWD) else P) + 7) // 8 * 8
            for m in modes}
    cpads = {m: ((P if m in (L.PACK_CONV_DGRAD, L.PACK_CONV_S1_DGRAD, L.PACK_CONVT_FWD) else Q) + 7) // 8 * 8
             for m in modes}
    for step in range(3):
        outs = [ops.packed(cache, w, m, pads[m], cpads[m], dt) for m in modes]  # the forward's operands
        gw, gb = _gen((P, Q, 4, 4), 100 + step), _gen((P,), 200 + step)
        w.grad, b.grad = gw.to(DEV), gb.to(DEV)
        ref_w.grad, ref_b.grad = gw.clone(), gb.clone()
        opt.step()
        ropt.step()
        torch.testing.assert_close(w.detach().cpu(), ref_w.detach(), rtol=0, atol=1e-6)
        torch.testing.assert_close(b.detach().cpu(), ref_b.detach(), rtol=0, atol=1e-6)
        for m, out in zip(modes, outs):
            fresh = ops.packed(cache, w, m, pads[m], cpads[m], dt)  # no repack if the step wrote it
            want = ops.pack(m, w, pads[m], cpads[m], dt)
            assert torch.equal(fresh.view(torch.int16 if dt == torch.bfloat16 else torch.int32),
                               want.view(torch.int16 if dt == torch.bfloat16 else torch.int32)), (step, m)
            if modes.index(m) < 2:
                assert fresh.data_ptr() == out.data_ptr()  # written in place by stc_adam_pack_step


def test_grad_accumulate_matches_add():
    """stc_grad_accumulate (the engine's sum of a network's real + fake weight gradients) == dst + src,
    bit-exact, for ragged sizes, misaligned (scalar-path) views and more than 16 tensors."""
    from stcgan_amd import ops
    g = torch.Generator(device="cuda").manual_seed(5)
    sizes = [1, 3, 4, 17, 4095, 4096, 4097, 65536 + 5, 1 << 20] + [257] * 12
    pairs, want = [], []
    for i, n in enumerate(sizes):
        d = torch.randn(n + 1, generator=g, device="cuda")
        s = torch.randn(n + 1, generator=g, device="cuda")
        if i % 3 == 1:  # 4-byte offset: the scalar path
            d, s = d[1:], s[1:]
        else:
            d, s = d[:n], s[:n]
        want.append(d + s)
        pairs.append((d, s))
    ops.grad_accumulate(pairs)
    for (d, _), w in zip(pairs, want):
        assert torch.equal(d, w)
