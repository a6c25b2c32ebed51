"""Cross-stream gradient hand-off of the side-stream step, under an adversarial schedule.

The trainer runs each discriminator on its own HIP stream (stcgan.STCGAN._on).  When a lane network's
output is read by several main-stream ops (the relativistic losses, STCGAN/stcgan.py:240-250, 280-290),
autograd sums the gradients those ops send back before handing them to the lane network's backward.
This test stalls the side stream (a device sleep enqueued on it) while the main stream, at the moment
the summed gradient is complete, allocates and fills scratch tensors of the same size -- the caching
allocator hands it the blocks autograd has just released -- and checks that the gradient the side
stream finally reads is still the right one.  (Round 3 probe: torch 2.10 sums and keeps these safely;
the trainer relies on it and this test pins it.)"""
import pytest
import torch

pytestmark = pytest.mark.gpu

N = 1 << 20
SLEEP_CYCLES = 200_000_000  # ~0.1 s of side-stream stall


class _OnStream(torch.autograd.Function):
    """A stand-in for a side-stream network (engine.NetFn): identity whose backward runs on the forward's
    stream, records the incoming gradient there and returns a copy computed on that stream."""

    @staticmethod
    def forward(ctx, x):
        return x * 1.0

    @staticmethod
    def backward(ctx, g):
        g.record_stream(torch.cuda.current_stream())
        return g * 1.0


def schedule():
    """x.grad of z = sum(2y) + sum(3y), y = _OnStream(x) on a side stream (expected: 5 everywhere)."""
    main = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    x = torch.ones(N, device="cuda", requires_grad=True)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        y = _OnStream.apply(x)
    y.record_stream(main)
    z = (y * 2.0).sum() + (y * 3.0).sum()
    junk = []

    def scribble(g):
        # the gradient of y is complete (both uses summed): overwrite whatever the main stream may reuse
        with torch.cuda.stream(main):
            for _ in range(8):
                junk.append(torch.full((N,), 1e6, device="cuda"))
        return None

    y.register_hook(scribble)
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        torch.cuda._sleep(SLEEP_CYCLES)
    z.backward()
    torch.cuda.synchronize()
    return float((x.grad - 5.0).abs().max())


def test_multi_use_gradient_sum_across_streams_under_stall():
    assert schedule() == 0.0
