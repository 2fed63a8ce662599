"""The committed golden fixtures are reproducible from the oracle (tools/make_golden.py),
and internally consistent.  GPU parity against them is in test_gpu_parity.py."""
import os

import numpy as np
import pytest

from tools import make_golden

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("name", ["my_scene_64.npz", "bench_128.npz", "forest_64.npz", "synth_small.npz",
                                  "spp_small.npz"])
def test_fixture_regenerates_bit_for_bit(name):
    committed = np.load(os.path.join(GOLDEN, name))
    fresh = make_golden.FIXTURES[name]()
    assert sorted(committed.files) == sorted(fresh)
    for k in committed.files:
        a, b = committed[k], fresh[k]
        assert a.dtype == b.dtype and a.shape == b.shape, k
        assert np.array_equal(a.view(np.uint8), np.ascontiguousarray(b).view(np.uint8)), k


def test_fixture_counters_consistent():
    g = np.load(os.path.join(GOLDEN, "my_scene_64.npz"))
    for d in (1, 2, 4, 8):
        node, shadow, pixels = g[f"counters_d{d}"]
        assert pixels == 64 * 64
        assert shadow % 3 == 0  # three point lights per hit
    # deeper recursion only adds rays
    assert g["counters_d8"][0] >= g["counters_d4"][0] >= g["counters_d2"][0] >= g["counters_d1"][0]
    # depth 1 == primary rays only
    assert g["counters_d1"][0] == 64 * 64
