"""Closed-form fixture weights and summaries shared by the golden generator and the tests.

TEST INFRASTRUCTURE ONLY.  The golden generator (``make_goldens.py``) loads
these weights into the *reference* networks; the tests regenerate the same
weights on any host from the same seeds (torch CPU ``Generator`` is
deterministic for a given torch build) and check them against the checksum
stored in each fixture before trusting a comparison.

Two weight families:
  * ``"ref"`` -- the distribution of ``weights_init`` in
    ``STCGAN/networks.py:9-20``: conv/convT/BN weight ~ N(0, 0.02), biases 0.
    (BN gamma ~ 0 makes outputs tiny; used for the train-step goldens because
    that is what the reference trains from.)
  * ``"one"`` -- BN gamma ~ N(1, 0.02), beta ~ N(0, 0.1), conv biases
    ~ N(0, 0.1): outputs span most of the tanh range, so a parity check is not
    vacuous.
Running statistics are always randomised (mean ~ N(0, 0.1), var ~ U(0.5, 1.5)) so
eval-mode batch-norm is exercised away from the identity.
"""
from collections import OrderedDict

import numpy as np
import torch


def fixture_state(template, seed, family="one"):
    """Return an OrderedDict with the keys/shapes of ``template`` filled deterministically."""
    g = torch.Generator().manual_seed(int(seed))
    out = OrderedDict()
    for name, t in template.items():
        shape = tuple(t.shape)
        if name.endswith("num_batches_tracked"):
            out[name] = torch.zeros((), dtype=torch.long)
        elif name.endswith("running_mean"):
            out[name] = torch.randn(shape, generator=g) * 0.1
        elif name.endswith("running_var"):
            out[name] = torch.rand(shape, generator=g) + 0.5
        elif name.endswith("weight") and len(shape) == 4:
            out[name] = torch.randn(shape, generator=g) * 0.02
        elif name.endswith("weight"):  # batch-norm gamma
            if family == "one":
                out[name] = 1.0 + torch.randn(shape, generator=g) * 0.02
            else:
                out[name] = torch.randn(shape, generator=g) * 0.02
        elif name.endswith("bias"):
            if family == "one":
                out[name] = torch.randn(shape, generator=g) * 0.1
            else:
                out[name] = torch.zeros(shape)
        else:
            raise KeyError(name)
    return out


def state_checksum(state):
    """float64 sum of |v| over every floating tensor, in key order."""
    s = 0.0
    for k, v in state.items():
        if v.is_floating_point():
            s += float(v.double().abs().sum())
    return s


def uniform(shape, seed, lo=-1.0, hi=1.0):
    g = torch.Generator().manual_seed(int(seed))
    return torch.rand(shape, generator=g) * (hi - lo) + lo


def pm_one(shape, seed):
    g = torch.Generator().manual_seed(int(seed))
    return (torch.rand(shape, generator=g) < 0.5).float() * 2.0 - 1.0


def normal(shape, seed):
    g = torch.Generator().manual_seed(int(seed))
    return torch.randn(shape, generator=g)


FULL_LIMIT = 65536
N_SAMPLES = 512


def sample_index(numel, key):
    seed = sum(ord(c) * (i + 1) for i, c in enumerate(key)) % (2 ** 31)
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, numel, (N_SAMPLES,), generator=g)


def put(d, key, t, limit=None):
    """Store a tensor fully if small, else a summary (sum, |sum|, sum^2, fixed samples)."""
    t = t.detach().cpu()
    if t.numel() <= (FULL_LIMIT if limit is None else limit) or not t.is_floating_point():
        d[key] = t.numpy().copy()  # copy: a later in-place update must not alias the fixture
        return
    f = t.double().reshape(-1)
    idx = sample_index(f.numel(), key)
    d[key + "::shape"] = np.array(t.shape, dtype=np.int64)
    d[key + "::sum"] = np.array(float(f.sum()))
    d[key + "::abssum"] = np.array(float(f.abs().sum()))
    d[key + "::sqsum"] = np.array(float((f * f).sum()))
    d[key + "::idx"] = idx.numpy()
    d[key + "::val"] = t.reshape(-1)[idx].numpy()


def compare(d, key, t, atol, rtol=0.0):
    """Compare tensor ``t`` against entry ``key`` of fixture ``d``; return max-abs error."""
    t = t.detach().cpu()
    if key in d:
        ref = torch.from_numpy(np.asarray(d[key]))
        assert tuple(ref.shape) == tuple(t.shape), (key, ref.shape, t.shape)
        if not t.is_floating_point():
            assert torch.equal(ref, t), key
            return 0.0
        err = (t.double() - ref.double()).abs()
        lim = atol + rtol * ref.double().abs()
        assert bool((err <= lim).all()), f"{key}: max err {float(err.max()):.3e}"
        return float(err.max())
    shape = tuple(int(s) for s in d[key + "::shape"])
    assert shape == tuple(t.shape), (key, shape, t.shape)
    f = t.double().reshape(-1)
    n = f.numel()
    vals = torch.from_numpy(np.asarray(d[key + "::val"])).double()
    idx = torch.from_numpy(np.asarray(d[key + "::idx"]))
    err = float((f[idx] - vals).abs().max())
    assert err <= atol + rtol * float(vals.abs().max()), f"{key} samples: {err:.3e}"
    s_ref = float(d[key + "::sum"])
    a_ref = float(d[key + "::abssum"])
    q_ref = float(d[key + "::sqsum"])
    assert abs(float(f.sum()) - s_ref) <= atol * n ** 0.5 * 4 + rtol * a_ref, key + "::sum"
    assert abs(float(f.abs().sum()) - a_ref) <= atol * n + rtol * a_ref, key + "::abssum"
    assert abs(float((f * f).sum()) - q_ref) <= (atol * 4) * float(f.abs().sum()) + rtol * q_ref * 2 + 1e-12, \
        key + "::sqsum"
    return err


def golden_rms(d, key):
    """Root-mean-square of fixture entry ``key`` (full tensor or summary): a scale for tolerances."""
    if key in d:
        a = np.asarray(d[key], dtype=np.float64)
        return float(np.sqrt((a * a).mean())) if a.size else 0.0
    n = int(np.prod(d[key + "::shape"]))
    return float(np.sqrt(float(d[key + "::sqsum"]) / max(n, 1)))


def compare_rel(d, key, t, rel):
    """compare() with the tolerance scaled by the golden's RMS: atol = rel * rms(golden)."""
    return compare(d, key, t, atol=rel * golden_rms(d, key) + 1e-12)
