"""The ray-queue radix sort (rust_tracer_amd/csrc/rt_order.hip) on its own.

Queue order never changes a frame (every task carries its parent slot, every shadow entry
its node and light), so the frame tests cannot see an unsorted queue -- only a lost or
duplicated entry.  These tests check the sort itself: for every digit width (8-bit
digits as in round 1, up to the 11-bit digits that sort 17- to 22-bit keys in two passes)
the values come out in stable key order, exactly numpy's stable argsort, including
ragged tails, one-digit inputs and keys with bits above `bits` (ignored by the sort).
"""
import ctypes as C

import numpy as np
import pytest
import torch

from rust_tracer_amd import abi

pytestmark = pytest.mark.gpu


def _sort(keys, bits, max_digit, vals=None):
    L = abi.lib()
    f = L.rt_debug_sort
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]
    dev = torch.device("cuda", 0)
    k = torch.from_numpy(keys.view(np.int32)).to(dev)
    v = torch.from_numpy(vals.view(np.int32)).to(dev) if vals is not None else None
    out = torch.full((len(keys),), -1, dtype=torch.int32, device=dev)
    rc = f(k.data_ptr(), v.data_ptr() if v is not None else None, len(keys), bits, max_digit, out.data_ptr())
    assert rc == 0, abi.STATUS_NAMES.get(rc, rc)
    return out.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("bits,max_digit", [(16, 8), (16, 11), (17, 8), (17, 11), (18, 11), (20, 11),
                                            (21, 11), (21, 8), (22, 11), (24, 11), (9, 11)])
@pytest.mark.parametrize("n", [1, 4095, 4097, 300_001])
def test_radix_sort_is_stable_argsort(bits, max_digit, n):
    rng = np.random.default_rng(bits * 1000 + n)
    keys = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    # clustered keys as the queues hold them: many repeats of few values
    keys[: n // 2] = (rng.integers(0, 37, size=n // 2) * 7919).astype(np.uint32)
    rng.shuffle(keys)
    got = _sort(keys, bits, max_digit)
    want = np.argsort(keys & np.uint32((1 << bits) - 1), kind="stable").astype(np.uint32)
    assert np.array_equal(got, want)


def test_radix_sort_carries_values():
    rng = np.random.default_rng(5)
    n = 1_000_003
    keys = rng.integers(0, 1 << 21, size=n).astype(np.uint32)
    vals = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    got = _sort(keys, 21, 11, vals)
    assert np.array_equal(got, vals[np.argsort(keys, kind="stable")])


def test_radix_sort_single_digit_value():
    keys = np.full(10_000, 0x1ABC, dtype=np.uint32)
    got = _sort(keys, 17, 11)
    assert np.array_equal(got, np.arange(10_000, dtype=np.uint32))
