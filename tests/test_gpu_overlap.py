"""The optimiser overlapped with the backward (STCGAN(args.overlap_optim=True), optim.Adam.overlap: each
gradient bucket updated on a side stream as soon as the backward completes it) must leave the trainer
bit-identical to the update-after-backward step: every parameter, BatchNorm buffer and Adam moment, over
several steps (the first steps take the general path, later ones the per-bucket launches), for both loss
families (the discriminators' buckets complete only after their second backward call)."""
import types

import pytest
import torch

pytestmark = pytest.mark.gpu

NETS = ("G1", "G2", "D1", "D2")


def _trainer(overlap, loss_type, dtype):
    from stcgan_amd.stcgan import STCGAN
    torch.manual_seed(11)
    a = types.SimpleNamespace(devices=["cuda:0"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5, beta2=0.999,
                              D_loss_fn="standard", D_loss_type=loss_type, ngf=16, dtype=dtype,
                              load_weights_g1=None, load_weights_g2=None, load_weights_d1=None,
                              load_weights_d2=None, overlap_optim=overlap, bucket_mb=0.25)
    return STCGAN(a)


@pytest.mark.parametrize("loss_type,dtype", [("normal", "bf16"), ("rel_avg", "fp32")])
def test_overlapped_update_is_bit_identical(loss_type, dtype):
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    B = 4
    x = torch.rand((B, 3, 256, 256), generator=g, device="cuda") * 2 - 1
    m = (torch.rand((B, 1, 256, 256), generator=g, device="cuda") < 0.5).float() * 2 - 1
    y = torch.rand((B, 3, 256, 256), generator=g, device="cuda") * 2 - 1
    a, b = _trainer(True, loss_type, dtype), _trainer(False, loss_type, dtype)
    for _ in range(4):
        a.train_step(x, m, y)
        b.train_step(x, m, y)
    assert len(a.optim_G._fast) == len(a.optim_D._fast) == 1  # the steady-state path ran
    assert a.optim_G._ov_stream is not None and a.optim_D._ov_stream is not None  # ... with per-bucket launches
    torch.cuda.synchronize()
    for n in NETS:
        sa, sb = getattr(a, n).state_dict(), getattr(b, n).state_dict()
        for k in sa:
            assert torch.equal(sa[k], sb[k]), (n, k)
    for on in ("optim_G", "optim_D"):
        oa, ob = getattr(a, on), getattr(b, on)
        for pa, pb in zip((p for g_ in oa.param_groups for p in g_["params"]),
                          (p for g_ in ob.param_groups for p in g_["params"])):
            assert torch.equal(oa.state[pa]["exp_avg"], ob.state[pb]["exp_avg"])
            assert torch.equal(oa.state[pa]["exp_avg_sq"], ob.state[pb]["exp_avg_sq"])
            assert float(oa.state[pa]["step"]) == float(ob.state[pb]["step"]) == 4.0
