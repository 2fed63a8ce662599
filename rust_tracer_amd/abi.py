"""ctypes mirror of include/rt_api.h (the C-ABI drop-in boundary).

Only data types and the loader for the product library live here.  The library is
``rust_tracer_amd/librt_hip.so`` (built in-tree by ``__graft_entry__.build()``); there is
no CPU fallback: if it is missing, :func:`lib` raises.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RT_LIB") or os.path.join(HERE, "librt_hip.so")  # RT_LIB: A/B tooling

RT_OK = 0
STATUS_NAMES = {
    0: "RT_OK", 1: "RT_ERR_INVALID_ARG", 2: "RT_ERR_SINGULAR_MATRIX",
    3: "RT_ERR_UNSUPPORTED", 4: "RT_ERR_NO_DEVICE", 5: "RT_ERR_HIP",
    6: "RT_ERR_OUT_OF_MEMORY", 7: "RT_ERR_BAD_MATERIAL", 8: "RT_ERR_CAPACITY",
}
RT_ERR_INVALID_ARG = 1
RT_ERR_UNSUPPORTED = 3
RT_ERR_NO_DEVICE = 4
RT_ERR_CAPACITY = 8
RT_MAX_DEPTH = 1024

RT_TEX_CONST, RT_TEX_CHECKERBOARD = 0, 1
RT_MAT_PHONG, RT_MAT_TEXTURE_PHONG = 0, 1
RT_SHAPE_SPHERE, RT_SHAPE_PLANE, RT_SHAPE_TRIANGLE, RT_SHAPE_CUBE = 0, 1, 2, 3
RT_LIGHT_POINT, RT_LIGHT_AMBIENT = 0, 1


class rt_color(C.Structure):
    _fields_ = [("r", C.c_float), ("g", C.c_float), ("b", C.c_float)]


class rt_texture(C.Structure):
    _fields_ = [("kind", C.c_int32), ("color", rt_color)]


class rt_material(C.Structure):
    _fields_ = [("kind", C.c_int32), ("ambient", rt_texture), ("diffuse", rt_texture),
                ("specular", rt_texture), ("power", C.c_float), ("reflectivity", C.c_float),
                ("refraction_index", C.c_float)]


class rt_shape(C.Structure):
    _fields_ = [("kind", C.c_int32), ("material", C.c_int32),
                ("transform", C.c_float * 16), ("data", C.c_float * 9)]


class rt_light(C.Structure):
    _fields_ = [("kind", C.c_int32), ("pos", C.c_float * 3), ("color", rt_color)]


class rt_scene_desc(C.Structure):
    _fields_ = [("n_materials", C.c_uint32), ("materials", C.POINTER(rt_material)),
                ("n_shapes", C.c_uint32), ("shapes", C.POINTER(rt_shape)),
                ("n_lights", C.c_uint32), ("lights", C.POINTER(rt_light)),
                ("ambient", rt_color)]


class rt_camera(C.Structure):
    _fields_ = [("origin", C.c_float * 3), ("x_min", C.c_float), ("x_max", C.c_float),
                ("y_min", C.c_float), ("y_max", C.c_float),
                ("x_res", C.c_uint32), ("y_res", C.c_uint32)]


class rt_counters(C.Structure):
    _fields_ = [("node_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("pixels", C.c_uint64),
                ("wave_iterations", C.c_uint64)]


class rt_render_opts(C.Structure):
    _fields_ = [("device", C.c_int32), ("counters", C.POINTER(rt_counters)),
                ("kernel_ms", C.POINTER(C.c_float))]


class rt_synth_params(C.Structure):
    """include/rt_scenes.h: the seeded synthetic scene of SURVEY.md §8(d)."""
    _fields_ = [("seed", C.c_uint64), ("n_spheres", C.c_uint32), ("n_cubes", C.c_uint32),
                ("n_triangles", C.c_uint32), ("r_min", C.c_float), ("r_max", C.c_float)]


def camera(x_res, y_res):
    """Camera::new (src/render.rs:166-176): origin (0,0,-8), window [-3,3]^2."""
    c = rt_camera()
    c.origin[:] = (0.0, 0.0, -8.0)
    c.x_min, c.x_max, c.y_min, c.y_max = -3.0, 3.0, -3.0, 3.0
    c.x_res, c.y_res = x_res, y_res
    return c


class RtError(RuntimeError):
    def __init__(self, status, what=""):
        super().__init__(f"{what}: {STATUS_NAMES.get(status, status)}")
        self.status = status


_lib = None


def lib():
    """Load librt_hip.so (the HIP product library).  Raises if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run __graft_entry__.build() "
                           "(the render path has no CPU fallback)")
    # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64.so.7 /
    # libhsa-runtime64.  Importing torch first makes our library bind to that already
    # loaded runtime (same soname), so torch.cuda / torch.distributed (RCCL) and the
    # render kernels share one HSA instance.  Loaded the other way round, torch finds
    # no GPU.  torch is optional: without it the system ROCm runtime is used.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    L = C.CDLL(LIB_PATH)
    P = C.POINTER
    vp = C.c_void_p
    L.rt_scene_create.argtypes = [P(rt_scene_desc), C.c_int32, P(vp)]
    L.rt_scene_create_tuned.argtypes = [P(rt_scene_desc), C.c_int32, C.c_char_p, P(vp)]
    L.rt_scene_set_tuning.argtypes = [vp, C.c_char_p]
    L.rt_scene_layout_digest.argtypes = [P(rt_scene_desc), C.c_char_p, P(C.c_uint64), P(C.c_uint64)]
    L.rt_scene_destroy.argtypes = [vp]
    L.rt_render.argtypes = [vp, P(rt_camera), C.c_uint32, P(rt_render_opts),
                            P(C.c_float), P(C.c_uint8)]
    L.rt_render_bands_async.argtypes = [vp, P(rt_camera), C.c_uint32, C.c_uint32, C.c_uint32,
                                        C.c_uint32, vp, vp, vp]
    L.rt_render_spp.argtypes = [vp, P(rt_camera), C.c_uint32, C.c_uint32, C.c_uint32, P(rt_render_opts),
                                P(C.c_float), P(C.c_uint8)]
    L.rt_render_bands_spp_async.argtypes = [vp, P(rt_camera), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                            C.c_uint32, C.c_uint32, vp, vp, vp]
    L.rt_render_bands_batch_async.argtypes = [vp, P(rt_camera), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                              C.c_uint32, vp, vp, vp]
    L.rt_render_bands_ex_async.argtypes = [vp, P(rt_camera), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                           C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, vp, vp]
    L.rt_render_bands_direct_async.argtypes = [vp, P(rt_camera), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                               C.c_uint32, vp, vp, vp, vp]
    L.rt_render_frame_async.argtypes = [vp, P(rt_camera), C.c_uint32, vp, vp, vp, vp]
    L.rt_scene_sync_status.argtypes = [vp]
    L.rt_scene_clone.argtypes = [vp, C.c_int32, P(vp)]
    L.rt_scene_create_multi.argtypes = [P(rt_scene_desc), P(C.c_int32), C.c_uint32, P(vp)]
    L.rt_scene_device_count.argtypes = [vp]
    L.rt_scene_device_count.restype = C.c_int32
    L.rt_scene_uses_rccl.argtypes = [vp]
    L.rt_scene_uses_rccl.restype = C.c_int32
    L.rt_unpermute_bands_u8_async.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp]
    for f in (L.rt_unpermute_bands_batch_async, L.rt_unpermute_bands_batch_u8_async):
        f.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp]
    L.rt_band_rows_per_rank.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
    L.rt_band_rows_per_rank.restype = C.c_uint32
    L.rt_unpermute_bands_async.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                           vp, vp]
    L.rt_quantize_u8_async.argtypes = [vp, C.c_size_t, vp, vp]
    L.rt_scene_flops_per_scan.argtypes = [vp]
    L.rt_scene_flops_per_scan.restype = C.c_uint64
    L.rt_scene_device_bytes.argtypes = [vp]
    L.rt_scene_device_bytes.restype = C.c_uint64
    L.rt_scene_workspace_bytes.argtypes = [vp]
    L.rt_host_alloc.argtypes = [C.c_uint64, C.POINTER(vp)]
    L.rt_host_free.argtypes = [vp]
    L.rt_scene_workspace_bytes.restype = C.c_uint64
    L.rt_scene_scan_ops.argtypes = [vp, P(C.c_uint64), C.c_uint32, C.c_int32]
    L.rt_scene_set_scan_counting.argtypes = [vp, C.c_int32]
    L.rt_scene_set_grid_share.argtypes = [vp, C.c_int32]
    L.rt_forest_create.argtypes = [vp, P(rt_camera), C.c_uint32, P(vp)]
    L.rt_forest_destroy.argtypes = [vp]
    L.rt_forest_render.argtypes = [vp, P(C.c_float)]
    L.rt_forest_render_filter.argtypes = [vp, P(C.c_int32), C.c_uint32, P(C.c_float)]
    L.rt_forest_tree_sizes.argtypes = [vp, P(C.c_uint32)]
    L.rt_forest_trees_with.argtypes = [vp, C.c_int32, P(C.c_uint64)]
    L.rt_forest_counters.argtypes = [vp, P(rt_counters)]
    L.rt_forest_timings.argtypes = [vp, P(C.c_float), P(C.c_float)]
    L.rt_scene_set_kernel_timing.argtypes = [vp, C.c_int32]
    L.rt_scene_kernel_times.argtypes = [vp, P(C.c_float), C.c_uint32, C.c_int32]
    L.rt_scene_set_material.argtypes = [vp, C.c_uint32, P(rt_material)]
    L.rt_scene_update.argtypes = [vp, P(rt_scene_desc), P(C.c_int32)]
    L.rt_write_image.argtypes = [C.c_char_p, P(C.c_uint8), C.c_uint32, C.c_uint32]
    L.rt_scene_uses_bvh.argtypes = [vp]
    L.rt_scene_uses_bvh.restype = C.c_int32
    L.rt_status_str.argtypes = [C.c_int32]
    L.rt_status_str.restype = C.c_char_p
    L.rt_api_version.restype = C.c_int32
    L.rt_max_frames.restype = C.c_uint32
    # scene builders (include/rt_scenes.h)
    L.rt_desc_my_scene.argtypes = [P(P(rt_scene_desc))]
    L.rt_desc_bench_128.argtypes = [P(P(rt_scene_desc))]
    L.rt_desc_synth.argtypes = [P(rt_synth_params), P(P(rt_scene_desc))]
    L.rt_desc_free.argtypes = [P(rt_scene_desc)]
    L.rt_synth_config.argtypes = [C.c_int32, P(rt_synth_params)]
    L.rt_mirror_render_calls.argtypes = [C.c_int32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int32,
                                         C.c_int32, P(C.c_float), P(C.c_int32), P(C.c_float), P(C.c_float)]
    _lib = L
    return L


def check(status, what=""):
    if status != RT_OK:
        raise RtError(status, what)
