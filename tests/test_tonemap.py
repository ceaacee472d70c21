"""hw5 Photographic tone mapping (pages/Page5.md:47-53 describes a global
operator, src/ has no code).  CPU: the oracle's restatement against closed forms; GPU:
rtg_tonemap against the oracle."""
import numpy as np
import pytest

import pyoracle
import rtg


def _gray(v, h=6, w=9):
    return np.full((h, w, 3), v, np.float32)


def test_constant_gray_maps_to_white():
    """A uniform gray image: L = key * Y / (Y + 1e-5) ~ key = Lwhite (burn 0), so Ld = 1."""
    out = pyoracle.tonemap(_gray(3.0), key=0.18, burn=0.0, gamma=2.2)
    assert np.allclose(out, 255.0, atol=1e-3)


def test_reinhard_curve_without_white_point():
    """burn 100 picks the darkest pixel as Lwhite (0 here): Ld = L / (1 + L), gamma 1."""
    img = np.zeros((4, 4, 3), np.float32)
    img[0, 0] = 10.0
    img[1, 1] = 2.0
    out = pyoracle.tonemap(img, key=0.5, burn=100.0, saturation=1.0, gamma=1.0)
    n = 16
    lw = np.exp((np.log(1e-5 + 10.0) + np.log(1e-5 + 2.0) + 14 * np.log(1e-5)) / n)
    for y, v in ((0, 10.0), (1, 2.0)):
        L = np.float32(0.5 / lw) * np.float32(v)
        assert abs(out[y, y, 0] - 255.0 * min(1.0, L / (1 + L))) < 1e-3
    assert out[2, 2].max() == 0.0


def test_saturation_and_monotonicity():
    rng = np.random.default_rng(5)
    img = (rng.random((20, 30, 3)) ** 3 * 50).astype(np.float32)
    out = pyoracle.tonemap(img, key=0.18, burn=2.0, saturation=0.5)
    assert np.isfinite(out).all() and out.min() >= 0 and out.max() <= 255
    y = (0.2126 * img[..., 0] + 0.7152 * img[..., 1]) + 0.0722 * img[..., 2]
    g = pyoracle.tonemap(np.repeat(y[..., None], 3, 2).astype(np.float32), key=0.18, burn=2.0)
    order = np.argsort(y.ravel())
    assert (np.diff(g[..., 0].ravel()[order]) >= -1e-3).all()      # monotone in luminance


@pytest.mark.gpu
@pytest.mark.parametrize("shape,burn,sat,gamma", [((1080, 1920), 1.0, 1.0, 2.2), ((37, 53), 0.0, 0.7, 1.8),
                                                  ((64, 64), 100.0, 1.2, 2.4)])
def test_gpu_tonemap_matches_oracle(gpu, shape, burn, sat, gamma):
    rng = np.random.default_rng(7)
    img = (rng.random(shape + (3,)) ** 4 * 1000).astype(np.float32)
    img[0, :5] = [[0, 0, 0], [np.nan, 1, 1], [np.inf, 0, 0], [-5, 2, 2], [1e30, 1e30, 1e30]]
    got = rtg.tonemap(img, key=0.18, burn=burn, saturation=sat, gamma=gamma, device=gpu)
    ref = pyoracle.tonemap(img, key=0.18, burn=burn, saturation=sat, gamma=gamma)
    assert np.isfinite(got).all()
    assert np.abs(got.astype(np.float64) - ref).max() < 1e-3
