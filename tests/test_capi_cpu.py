"""CPU-only checks of the C-ABI library and the host logic (no GPU compute)."""
import ctypes
import os
import re

import pytest
import torch

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "stcgan_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(stc_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from stcgan_amd import _lib
    h = ctypes.CDLL(_lib.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(h, s)]
    assert not missing, missing
    # and the Python binding covers exactly the declared surface
    assert sorted(_lib.EXPORTED) == syms


def test_library_host_queries():
    from stcgan_amd import _lib
    lib = _lib.lib()
    assert lib.stc_version() >= 1
    assert lib.stc_adam_elems_per_block() == 1024
    assert 1 <= lib.stc_chan_stats_chunks(32, 128, 128) <= 1024
    assert lib.stc_loss_parts(1) == 1
    # split-K workspace sizes: big-M layers need none, the bottleneck needs slabs
    assert lib.stc_conv_fwd_workspace(0, 0, 32, 64, 64, 64, 128) == 0
    assert lib.stc_conv_fwd_workspace(0, 0, 32, 2, 2, 512, 512) > 0
    assert lib.stc_conv_wgrad_workspace(0, 32, 64, 64, 128, 64) > 0


def test_invalid_arguments_fail_loudly_without_gpu():
    """Argument validation happens before any launch: the error text comes back through stc_last_error."""
    from stcgan_amd import _lib
    lib = _lib.lib()
    v = _lib.View(None, 4, 4, 0, 0, 3, 0, 1, 0)
    rc = lib.stc_conv_fwd(0, 0, 1, v, 3, None, None, 0, 0.0, None, 8, v, None, 0, 1, None, 0, None)
    assert rc != 0
    assert b"Cin=3" in lib.stc_last_error()
    with pytest.raises(RuntimeError, match="must be a multiple of 4"):
        _lib.check(rc, "stc_conv_fwd")


@pytest.mark.parametrize("name,in_c,out_c", [("G1", 3, 1), ("G2", 4, 3)])
def test_generator_module_tree_matches_reference(name, in_c, out_c):
    from oracle import stcgan_ref as ref
    from stcgan_amd import networks
    for ngf in (8, 64):
        net = networks.get_generator(in_c, out_c, ngf=ngf)
        tmpl = ref.generator_state_template(in_c, out_c, ngf)
        sd = net.state_dict()
        assert list(sd) == list(tmpl)
        assert all(tuple(sd[k].shape) == tuple(tmpl[k].shape) for k in sd)


@pytest.mark.parametrize("in_c", [4, 7])
def test_discriminator_module_tree_matches_reference(in_c):
    from oracle import stcgan_ref as ref
    from stcgan_amd import networks
    net = networks.get_discriminator(in_c, ndf=64, n_layers=3, use_sigmoid=False)
    tmpl = ref.discriminator_state_template(in_c, 64)
    assert list(net.state_dict()) == list(tmpl)


def test_reference_checkpoint_loads(tmp_path):
    """A state_dict saved from the oracle template (same keys as the reference's .pt files) loads strictly."""
    from oracle import stcgan_ref as ref
    from stcgan_amd import networks
    from fixture_init import fixture_state
    st = fixture_state(ref.generator_state_template(3, 1, 8), 5, "ref")
    p = tmp_path / "G1-latest.pt"
    torch.save(st, p)
    net = networks.get_generator(3, 1, ngf=8)
    net.load_state_dict(torch.load(p, weights_only=True))
    for k, v in net.state_dict().items():
        assert torch.equal(v, st[k])


def test_forward_on_cpu_fails_loudly():
    from stcgan_amd import networks
    net = networks.get_generator(3, 1, ngf=8)
    with pytest.raises(RuntimeError, match="GPU only"):
        net(torch.zeros(1, 3, 256, 256))


def test_generator_plan_and_sizes():
    from stcgan_amd import engine, networks
    net = networks.get_generator(4, 3, ngf=8)
    plan = engine.GenPlan(net)
    assert plan.L == 8 and plan.in_c == 4 and plan.out_c == 3
    assert plan.co == [8, 16, 32, 64, 64, 64, 64, 64]
    assert len(plan.bnd) == 6 and len(plan.bnu) == 7
    # 480x640: the pad/crop levels of src/models/stcgan_g.py (15x20 -> 16x20, 4x5 -> 4x6)
    S = engine._sizes(480, 640, 8)
    assert S[:9] == [(480, 640), (240, 320), (120, 160), (60, 80), (30, 40), (15, 20), (8, 10), (4, 5), (2, 3)]
    assert engine._pad2(S, 5) == (16, 20) and engine._pad2(S, 7) == (4, 6)


def test_discriminator_plan():
    from stcgan_amd import engine, networks
    net = networks.get_discriminator(7, ndf=64)
    plan = engine.DiscPlan(net)
    assert plan.strides == [2, 2, 2, 1, 1] and plan.in_c == 7
    assert [c.out_channels for c in plan.convs] == [64, 128, 256, 512, 1]


def test_flop_count_matches_survey():
    import bench
    f = bench.gen_fwd_flops(3, 1, 64, 32, 256, 256) + bench.gen_fwd_flops(4, 3, 64, 32, 256, 256)
    assert abs(f / 1e9 - 770.95) < 0.01  # SURVEY.md section 8d / BASELINE.md


def test_channel_padding_rules():
    from stcgan_amd import ops
    assert ops.pad_channels(3, torch.float32) == 4
    assert ops.pad_channels(7, torch.float32) == 8
    assert ops.pad_channels(3, torch.bfloat16) == 8
    assert ops.pad_channels(64, torch.bfloat16) == 64
