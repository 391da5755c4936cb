"""rm_sample_batch, the device batch sampler (SceneDataset::sample_batch, dataset.rs:47-82):
the uniform share draws every pixel with equal probability, the boost share only foreground
pixels, the rows are the gathered rows of those pixels (dataset.rs:75-79), and a batch is a
function of (seed, stream, counter) alone. The reference draws with an unseeded rand::rng(), so
the match is in distribution (chi-square bounds, stated per check)."""
import ctypes

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]


def _sample(torch, render, src, fg, nu, nf, seed, stream, counter):
    ctx = render.context()
    o, d, t = src
    n = nu + nf
    out = [torch.empty((n, 3), device="cuda") for _ in range(3)]
    idx = torch.empty(n, dtype=torch.int32, device="cuda")
    p = lambda x: ctypes.c_void_p(x.data_ptr()) if x is not None else None  # noqa: E731
    ctx.check(ctx._lib.rm_sample_batch(ctx.handle, p(o), p(d), p(t), o.shape[0], p(fg), 0 if fg is None else fg.numel(),
                                       nu, nf, seed, stream, counter, p(out[0]), p(out[1]), p(out[2]), p(idx)),
              "rm_sample_batch")
    torch.cuda.synchronize()
    return idx.cpu().numpy(), [x.cpu().numpy() for x in out]


def test_device_sampler():
    import torch
    from burn_raymarching_amd import render
    rng = np.random.default_rng(0)
    npix = 100_000
    host = [rng.normal(size=(npix, 3)).astype(np.float32) for _ in range(3)]
    src = [torch.from_numpy(h).cuda() for h in host]
    fg_np = np.sort(rng.choice(npix, 7_000, replace=False)).astype(np.int32)
    fg = torch.from_numpy(fg_np).cuda()
    nu, nf = 400_000, 100_000
    idx, (o, d, t) = _sample(torch, render, src, fg, nu, nf, 5, 1, 0)
    assert idx.min() >= 0 and idx.max() < npix
    # the gathered rows are the drawn pixels' rows, bit for bit
    for got, h in zip((o, d, t), host):
        assert np.array_equal(got, h[idx])
    # boost share: foreground only, every foreground pixel equally likely (chi-square, 99.99 %)
    assert np.isin(idx[nu:], fg_np).all()
    cnt = np.bincount(np.searchsorted(fg_np, idx[nu:]), minlength=fg_np.size)
    chi = ((cnt - nf / fg_np.size) ** 2 / (nf / fg_np.size)).sum()
    dof = fg_np.size - 1
    assert chi < dof + 4.5 * np.sqrt(2 * dof), chi
    # uniform share: 1000 equal buckets of the pixel range
    cnt = np.bincount(idx[:nu] * 1000 // npix, minlength=1000)
    chi = ((cnt - nu / 1000) ** 2 / (nu / 1000)).sum()
    assert chi < 999 + 4.5 * np.sqrt(2 * 999), chi
    # a function of (seed, stream, counter): same -> same, any change -> different batch
    again, _ = _sample(torch, render, src, fg, nu, nf, 5, 1, 0)
    assert np.array_equal(idx, again)
    for key in ((6, 1, 0), (5, 2, 0), (5, 1, 1)):
        other, _ = _sample(torch, render, src, fg, nu, nf, *key)
        assert (other != idx).mean() > 0.99
    # the first rows do not depend on the batch size (counter-based draws)
    short, _ = _sample(torch, render, src, fg, 1000, 0, 5, 1, 0)
    assert np.array_equal(short, idx[:1000])
    # no foreground: uniform draws only; zero rows: no launch
    only, _ = _sample(torch, render, src, None, 5000, 0, 1, 1, 1)
    assert only.shape == (5000,)
    ctx = render.context()
    rc = ctx._lib.rm_sample_batch(ctx.handle, None, None, None, npix, None, 0, 0, 10, 1, 1, 1, None, None, None,
                                  ctypes.c_void_p(src[0].data_ptr()))
    assert rc == 1  # n_fg > 0 without a foreground list
