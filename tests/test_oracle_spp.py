"""The oracle's supersampling (config 5, rt_render_spp's jitter; no reference equivalent,
SURVEY.md §7 step 6): spp = 1 is render.rs exactly, the jitter is a pure function of
(seed, pixel, sample), and the averaged frame stays an average of the same scene."""
import numpy as np

from oracle.oracle import OracleScene


def mix32(x):
    x = np.uint32(x)
    x ^= x >> np.uint32(16)
    x = np.uint32((int(x) * 0x7feb352d) & 0xFFFFFFFF)
    x ^= x >> np.uint32(15)
    x = np.uint32((int(x) * 0x846ca68b) & 0xFFFFFFFF)
    x ^= x >> np.uint32(16)
    return x


def jitter(seed, pixel, sample, dim):
    """include/rt_api.h rt_render_spp, restated"""
    h = mix32(mix32(seed ^ 0x9e3779b9) ^ np.uint32(pixel))
    h = mix32(h ^ mix32(2 * sample + dim + 1))
    return np.float32(int(h >> np.uint32(8))) * np.float32(1.0 / 16777216.0)


def test_spp1_is_render():
    o = OracleScene()
    a, ca = o.render(48, 40, 4)
    b, cb = o.render(48, 40, 4, spp=1, seed=7)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert ca == cb


def test_spp_counts_samples_and_is_deterministic():
    o = OracleScene()
    a, ca = o.render(32, 24, 3, spp=4, seed=3, threads=4)
    b, cb = o.render(32, 24, 3, spp=4, seed=3, threads=1)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and ca == cb
    assert ca["pixels"] == 32 * 24 * 4
    c, _ = o.render(32, 24, 3, spp=4, seed=4)
    assert not np.array_equal(a, c)  # the seed changes the samples


def test_supersampled_frame_is_an_average():
    o = OracleScene()
    one, _ = o.render(64, 64, 2)
    many, _ = o.render(64, 64, 2, spp=16, seed=3, threads=8)
    # same scene, same exposure: the mean colour moves by a fraction of a pixel's footprint
    assert abs(float(many.mean()) - float(one.mean())) < 0.02 * abs(float(one.mean())) + 1e-3
    # the samples are spread inside the pixel: jitter in [0, 1), roughly uniform
    js = np.array([jitter(3, p, k, d) for p in range(64) for k in range(16) for d in range(2)])
    assert js.min() >= 0.0 and js.max() < 1.0
    assert abs(js.mean() - 0.5) < 0.05
