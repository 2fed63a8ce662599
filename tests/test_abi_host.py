"""CPU-side checks of the drop-in boundary and the host logic (no GPU needed).

- librt_hip.so loads and exports every entry point include/*.h declares;
- rt_scene_create validates the description on the host (errors, not panics) before it
  touches a device; without a GPU it reports RT_ERR_NO_DEVICE;
- the C++ host mirror of the Scene API builds my_scene.rs exactly: rendered by the CPU
  oracle, its flattened description equals the oracle's own restatement bit for bit;
- Python Matrix composition == the oracle's matrix.rs restatement;
- row-band bookkeeping (the multi-GPU split) is a partition of the frame.
"""
import ctypes as C
import os
import re

import numpy as np
import pytest

import rust_tracer_amd as rt
from rust_tracer_amd import abi
from rust_tracer_amd.dist import band_rows_per_rank_py, local_rows

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in ("rt_api.h", "rt_scenes.h"):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^\s*(?:[A-Za-z_][\w\s\*]*?)\b(rt_\w+)\s*\(", text, flags=re.M):
            names.add(m.group(1))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    L = abi.lib()
    names = declared_functions()
    assert len(names) >= 15, names
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert L.rt_api_version() == 1
    assert L.rt_status_str(2) == b"RT_ERR_SINGULAR_MATRIX"


def test_no_cpu_render_path():
    """Without a HIP device the product refuses to render (no silent CPU fallback)."""
    from tests.conftest import gpu_available
    if gpu_available():
        pytest.skip("a GPU is present")
    with pytest.raises(rt.RtError) as e:
        rt.DeviceScene(rt.SceneDesc.my_scene())
    assert e.value.status == 4  # RT_ERR_NO_DEVICE


def _create(desc):
    h = C.c_void_p()
    return abi.lib().rt_scene_create(desc.ptr(), -1, C.byref(h))


def test_scene_create_validates_before_device():
    d = rt.SceneDesc()
    m = d.phong((0, 0, 0), (1, 1, 1), (1, 1, 1), 60, 0, 0)
    d.sphere(m, rt.Matrix.scale(0, 1, 1))  # singular: Matrix::invert panics in the reference
    assert _create(d) == 2
    d = rt.SceneDesc()
    d.sphere(5)  # material index out of range
    assert _create(d) == 7
    d = rt.SceneDesc()
    m = d.phong((0, 0, 0), (1, 1, 1), (1, 1, 1), 60, 0, 0)
    d.materials[0].diffuse.kind = abi.RT_TEX_CHECKERBOARD  # textures need TexturePhong
    d.sphere(m)
    assert _create(d) == 1


def test_rt_render_rejects_bad_arguments():
    L = abi.lib()
    cam = abi.camera(4, 4)
    rgb = (C.c_float * 48)()
    assert L.rt_render(None, C.byref(cam), 1, None, rgb, None) == 1
    assert L.rt_unpermute_bands_async(None, 4, 4, 8, 1, None, None) == 1
    assert L.rt_quantize_u8_async(None, 4, None, None) == 1
    buf = (C.c_float * 48)()
    # frame batches: n_frames within stride_frames, both > 0
    assert L.rt_unpermute_bands_batch_async(None, 4, 4, 8, 1, 1, 1, buf, None) == 1
    assert L.rt_unpermute_bands_batch_async(buf, 4, 4, 8, 1, 2, 1, buf, None) == 1
    assert L.rt_unpermute_bands_batch_async(buf, 4, 4, 8, 1, 0, 1, buf, None) == 1
    assert L.rt_unpermute_bands_batch_u8_async(None, 4, 4, 8, 1, 1, 1, None, None) == 1
    assert L.rt_scene_set_grid_share(None, 50) == 1


def test_host_my_scene_matches_oracle_restatement_bit_for_bit():
    """include/rt_scenes.h rt_desc_my_scene (C++ host mirror of my_scene.rs) rendered by
    the oracle == the oracle's own my_scene.rs restatement."""
    from oracle.oracle import OracleScene
    a, ca = OracleScene().render(96, 72, 8)
    b, cb = OracleScene(rt.SceneDesc.my_scene()).render(96, 72, 8)
    assert ca == cb
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_python_matrix_matches_oracle():
    from oracle import oracle as O
    L = O.lib()
    m = rt.Matrix.translate(-1.0, 0.0, 0.0) * rt.Matrix.rotate_z(75.0) * rt.Matrix.scale(1.0, 0.25, 1.0)
    a, b, c, out = (C.c_float * 16)(), (C.c_float * 16)(), (C.c_float * 16)(), (C.c_float * 16)()
    L.oracle_matrix_translate(-1.0, 0.0, 0.0, a)
    L.oracle_matrix_rotate_z(75.0, b)
    L.oracle_matrix_scale(1.0, 0.25, 1.0, c)
    L.oracle_matrix_mul(a, b, out)
    L.oracle_matrix_mul((C.c_float * 16)(*out), c, out)
    assert np.array_equal(np.array(out[:], np.float32), np.array(m.flat(), np.float32))


def test_synth_scenes_are_deterministic_and_sized():
    d2 = rt.SceneDesc.synth_config(2)
    d3 = rt.SceneDesc.synth_config(3)
    assert d2.n_shapes == 102
    assert d3.n_shapes == 600 + 25 + 100 + 2
    again = rt.SceneDesc.synth_config(3)
    s1 = d3.ptr().contents
    s2 = again.ptr().contents
    raw = lambda s: bytes(C.string_at(s.shapes, s.n_shapes * C.sizeof(abi.rt_shape)))
    assert raw(s1) == raw(s2)


@pytest.mark.parametrize("h,band,world", [(1080, 8, 1), (1080, 8, 2), (1080, 8, 8), (117, 8, 3),
                                          (7, 8, 4), (2160, 16, 8)])
def test_bands_partition_the_frame(h, band, world):
    L = abi.lib()
    rpr = band_rows_per_rank_py(h, band, world)
    assert rpr == L.rt_band_rows_per_rank(h, band, world)
    seen = []
    for r in range(world):
        rows = local_rows(h, band, r, world)
        assert len(rows) == rpr
        seen += [v for v in rows if v >= 0]
    assert sorted(seen) == list(range(h))


def test_multi_device_scene_needs_devices():
    """rt_scene_create_multi validates its device list; without a HIP device it reports
    RT_ERR_NO_DEVICE like rt_scene_create (no CPU fallback)."""
    from tests.conftest import gpu_available
    L = abi.lib()
    h = C.c_void_p()
    desc = rt.SceneDesc.my_scene()
    assert L.rt_scene_create_multi(desc.ptr(), None, 1, C.byref(h)) == 1  # RT_ERR_INVALID_ARG
    devs = (C.c_int32 * 2)(0, 1)
    assert L.rt_scene_create_multi(desc.ptr(), devs, 0, C.byref(h)) == 1
    if not gpu_available():
        assert L.rt_scene_create_multi(desc.ptr(), devs, 2, C.byref(h)) == 4  # RT_ERR_NO_DEVICE
    assert L.rt_scene_device_count(None) == 0
    assert L.rt_status_str(abi.RT_ERR_CAPACITY) == b"RT_ERR_CAPACITY"
    assert L.rt_scene_sync_status(None) == 1


def test_tuning_strings_are_validated_on_the_host():
    """rt_scene_create_tuned parses its tuning string (rt_tune.hpp) before it touches a
    device: an unknown key, a bad value or a malformed pair is RT_ERR_INVALID_ARG; a valid
    string gets as far as the device (RT_ERR_NO_DEVICE here).  The environment's RT_TUNE is
    parsed the same way."""
    L = abi.lib()
    desc = rt.SceneDesc.my_scene()
    h = C.c_void_p()
    gpu = L.rt_scene_create(desc.ptr(), 0, C.byref(h)) == abi.RT_OK
    if gpu:
        L.rt_scene_destroy(h)
        pytest.skip("a HIP device is present: the valid strings would create scenes")
    for bad in (b"bogus=1", b"lb_res", b"lb_res=x", b"task_w=48", b"sort=maybe", b"seam_split=0",
                b"shadow_key=17", b"=3", b"lb_tiers=0", b"lb_tiers=8", b"lb_dmax_k=0.5"):
        assert L.rt_scene_create_tuned(desc.ptr(), 0, bad, C.byref(h)) == abi.RT_ERR_INVALID_ARG, bad
    for good in (b"", b"lb_res=0,bvh=0", b"task_w=32 task_fill=2.5", b"sort=shadow,dup=shc",
                 b"shadow_key=cell,frame_keys=frame,spp_keys=mix", b"lds_nodes=trace,seam_adapt=device",
                 b"force_rccl=1,node_cap=4096", b"graze_k=3e-3,bvh_cnode=200,bvh_maxleaf=16",
                 b"lb_tiers=1", b"lb_tiers=7,lb_res=32", b"lb_dmax_k=2.01"):
        assert L.rt_scene_create_tuned(desc.ptr(), 0, good, C.byref(h)) == abi.RT_ERR_NO_DEVICE, good


def _layout_digest(desc, tuning):
    dg, nb = C.c_uint64(), C.c_uint64()
    st = abi.lib().rt_scene_layout_digest(desc.ptr(), tuning.encode(), C.byref(dg), C.byref(nb))
    assert st == 0, st
    return dg.value, nb.value


@pytest.mark.parametrize("which", ["my_scene", "config3", "stress"])
def test_scene_build_is_deterministic_over_host_threads(which):
    """rt_scene_create's host build (hierarchy, light-buffer tiers built by several host
    threads, shape buffers) produces the same device image for any thread count
    (rt_scene_layout_digest: the host half alone, no GPU)."""
    if which == "my_scene":
        desc = rt.SceneDesc.my_scene()
    elif which == "config3":
        desc = rt.SceneDesc.synth_config(3)
    else:
        from tests.test_gpu_cull_stress import stress_scene
        desc = stress_scene(13, 1000.0, False, True)
    one = _layout_digest(desc, "build_threads=1")
    assert one == _layout_digest(desc, "build_threads=5")
    assert one == _layout_digest(desc, "")
    assert one[1] > 0


def test_more_than_max_lights_are_refused_on_the_host():
    """rt_api.h RT_MAX_LIGHTS (65536: the shadow keys' 16-bit light index).  300 lights build
    (wide shadow entries past 256), 65537 are refused with RT_ERR_UNSUPPORTED before any device
    work (and before any light buffer is built)."""
    from tests.test_gpu_many_lights import _scene
    assert _layout_digest(_scene(256), "lb_res=4")[1] > 0
    assert _layout_digest(_scene(300), "lb_res=4")[1] > 0
    d = rt.SceneDesc()
    for k in range(65537):
        d.point_light((0.0, 10.0 + k * 1e-3, 0.0), (0.0, 0.0, 0.0))
    dg, nb = C.c_uint64(), C.c_uint64()
    st = abi.lib().rt_scene_layout_digest(d.ptr(), b"lb_res=4", C.byref(dg), C.byref(nb))
    assert st == abi.RT_ERR_UNSUPPORTED
