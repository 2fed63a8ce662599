"""The device path's powf (rust_tracer_amd/csrc/rt_powf.hpp) against the reference's: the
specular term m_dot_h.powf(power) (material.rs:211) is the platform libm's powf, which the
oracle calls (oracle.powf).  rt_powf.hpp replays glibc's own evaluation (double-precision
log2 / exp2 tables, FMA build), so every value must be bit-identical -- including the
overflow to inf that a scaled plane normal produces (tests/test_gpu_seam.py) and the
specials (0, 1, inf, NaN, negative bases, subnormals).

CPU: the same header compiled for the host (rt_powf_batch_host).  GPU: the kernel
(rt_powf_batch_async) -- the code the combine pass runs.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import oracle
from rust_tracer_amd import abi


def inputs(n=400_000, seed=5):
    rng = np.random.default_rng(seed)
    parts = []
    # the render's domain: m.h in [0, 1] (and a little above: scaled plane normals), powers
    for p in (60.0, 600.0, 500.0, 128.0, 1.0, 2.0, 0.5, 1e6):
        x = rng.random(n // 8, dtype=np.float32)
        parts.append((np.concatenate([x, 1 + x]), np.full(2 * x.size, p, np.float32)))
    # random bit patterns (every class of float) and integer / half-integer exponents
    bits = rng.integers(0, 2**32, size=(2, n), dtype=np.uint64).astype(np.uint32)
    parts.append((bits[0].view(np.float32), bits[1].view(np.float32)))
    xs = np.abs(bits[0].view(np.float32))
    parts.append((xs, (rng.integers(-400, 400, n) * 0.5).astype(np.float32)))
    sp = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 1.17e-38, 3.4e38, 0.5, 2.0, -2.0],
                  np.float32)
    gx, gy = np.meshgrid(sp, sp)
    parts.append((gx.ravel(), gy.ravel()))
    x = np.concatenate([p[0] for p in parts]).astype(np.float32)
    y = np.concatenate([p[1] for p in parts]).astype(np.float32)
    return x, y


def same(a, b):
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def test_host_build_bit_identical_to_libm():
    x, y = inputs()
    ref = oracle.powf(x, y)
    out = np.empty_like(x)
    f = C.POINTER(C.c_float)
    abi.check(abi.lib().rt_powf_batch_host(x.ctypes.data_as(f), y.ctypes.data_as(f), out.ctypes.data_as(f), x.size),
              "rt_powf_batch_host")
    ok = same(out, ref)
    bad = np.flatnonzero(~ok)[:5]
    assert ok.all(), [(float(x[i]), float(y[i]), float(out[i]), float(ref[i])) for i in bad]


@pytest.mark.gpu
def test_device_bit_identical_to_libm():
    import torch
    x, y = inputs(seed=9)
    ref = oracle.powf(x, y)
    dev = torch.device("cuda", 0)
    dx, dy = torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)
    dout = torch.empty_like(dx)
    st = torch.cuda.current_stream(dev).cuda_stream
    abi.check(abi.lib().rt_powf_batch_async(C.c_void_p(dx.data_ptr()), C.c_void_p(dy.data_ptr()),
                                            C.c_void_p(dout.data_ptr()), x.size, C.c_void_p(st)), "rt_powf_batch_async")
    out = dout.cpu().numpy()
    ok = same(out, ref)
    bad = np.flatnonzero(~ok)[:5]
    assert ok.all(), [(float(x[i]), float(y[i]), float(out[i]), float(ref[i])) for i in bad]
