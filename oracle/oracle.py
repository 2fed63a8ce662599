"""TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU oracle (oracle/liboracle.so).

The oracle is a C++ restatement of the reference render path (see oracle_api.h).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module;
the product (rust_tracer_amd) never does.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_lib = None


class oracle_hit(C.Structure):
    _fields_ = [("hit", C.c_int32), ("id", C.c_int32), ("t", C.c_float),
                ("point", C.c_float * 3), ("eye_dir", C.c_float * 3), ("normal", C.c_float * 3),
                ("entering", C.c_int32), ("tex", C.c_float * 2)]


def build():
    """Compile liboracle.so with the committed Makefile (g++, -ffp-contract=off)."""
    subprocess.run(["make", "-C", HERE, "-s"], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    from rust_tracer_amd import abi  # ctypes types of the shared data formats only
    L = C.CDLL(LIB_PATH)
    P, vp, f = C.POINTER, C.c_void_p, C.c_float
    fa = P(C.c_float)
    L.oracle_scene_from_desc.argtypes = [P(abi.rt_scene_desc), P(vp)]
    L.oracle_scene_my_scene.argtypes = [P(vp)]
    L.oracle_scene_destroy.argtypes = [vp]
    L.oracle_render_rows.argtypes = [vp, P(abi.rt_camera), C.c_uint32, C.c_uint32, C.c_uint32,
                                     C.c_uint32, fa, P(C.c_uint64)]
    L.oracle_render_rows_mt.argtypes = [vp, P(abi.rt_camera), C.c_uint32, C.c_uint32, C.c_uint32,
                                        C.c_uint32, fa, P(C.c_uint64), C.c_uint32]
    L.oracle_render_rows_spp_mt.argtypes = [vp, P(abi.rt_camera), C.c_uint32, C.c_uint32, C.c_uint32,
                                            C.c_uint32, C.c_uint32, C.c_uint32, fa, P(C.c_uint64), C.c_uint32]
    L.oracle_render_forest.argtypes = [vp, P(abi.rt_camera), C.c_uint32, fa, P(C.c_uint32)]
    L.oracle_forest_build.argtypes = [vp, P(abi.rt_camera), C.c_uint32, P(vp)]
    L.oracle_forest_render.argtypes = [vp, fa]
    L.oracle_forest_build_mt.argtypes = [vp, P(abi.rt_camera), C.c_uint32, C.c_uint32, P(vp)]
    L.oracle_forest_render_mt.argtypes = [vp, fa, C.c_uint32]
    L.oracle_forest_render_filter.argtypes = [vp, P(C.c_int32), C.c_uint32, fa]
    L.oracle_forest_tree_sizes.argtypes = [vp, P(C.c_uint32)]
    L.oracle_forest_trees_with.argtypes = [vp, C.c_int32]
    L.oracle_forest_trees_with.restype = C.c_uint64
    L.oracle_forest_destroy.argtypes = [vp]
    L.oracle_scene_set_material.argtypes = [vp, C.c_uint32, P(abi.rt_material)]
    L.oracle_as_u8.argtypes = [fa, C.c_uint64, P(C.c_uint8)]
    L.oracle_powf_batch.argtypes = [fa, fa, fa, C.c_uint64]
    L.oracle_libm_batch.argtypes = [C.c_int, fa, fa, fa, C.c_uint64]
    for n in ("identity",):
        getattr(L, "oracle_matrix_" + n).argtypes = [fa]
    for n in ("scale", "translate"):
        getattr(L, "oracle_matrix_" + n).argtypes = [f, f, f, fa]
    for n in ("rotate_x", "rotate_y", "rotate_z"):
        getattr(L, "oracle_matrix_" + n).argtypes = [f, fa]
    L.oracle_matrix_mul.argtypes = [fa, fa, fa]
    L.oracle_matrix_transpose.argtypes = [fa, fa]
    L.oracle_matrix_inverse.argtypes = [fa, fa]
    for n in ("oracle_matrix_pt_mul", "oracle_matrix_vec3_mul"):
        getattr(L, n).argtypes = [fa, fa, fa]
    for n in ("oracle_pt_mat_mul", "oracle_vec3_mat_mul"):
        getattr(L, n).argtypes = [fa, fa, fa]
    L.oracle_sphere_intersect.argtypes = [fa, fa, fa, P(oracle_hit)]
    L.oracle_triangle_normal.argtypes = [fa, fa, fa, fa]
    L.oracle_triangle_intersect.argtypes = [fa, fa, fa, fa, fa, P(oracle_hit)]
    L.oracle_plane_axes.argtypes = [fa, fa, fa]
    L.oracle_plane_intersect.argtypes = [fa, fa, fa, fa, fa, P(oracle_hit)]
    L.oracle_cube_intersect.argtypes = [fa, fa, fa, P(oracle_hit)]
    L.oracle_phong_reflected_energy.argtypes = [P(abi.rt_color)] * 3 + [f, P(abi.rt_color), fa,
                                                                         P(oracle_hit), P(abi.rt_color)]
    L.oracle_checkerboard.argtypes = [f, f, P(abi.rt_color)]
    L.oracle_fresnel_reflection.argtypes = [fa, fa, f, f]
    L.oracle_fresnel_reflection.restype = C.c_float
    _lib = L
    return L


def farr(vals, n=None):
    vals = list(vals)
    a = (C.c_float * (n or len(vals)))()
    a[:len(vals)] = [float(np.float32(v)) for v in vals]
    return a


class OracleScene:
    def __init__(self, desc=None):
        """desc: a rust_tracer_amd.SceneDesc, or None for the oracle's own my_scene.rs."""
        self.L = lib()
        self.h = C.c_void_p()
        if desc is None:
            st = self.L.oracle_scene_my_scene(C.byref(self.h))
        else:
            st = self.L.oracle_scene_from_desc(desc.ptr(), C.byref(self.h))
        if st != 0:
            raise RuntimeError(f"oracle scene construction failed: status {st}")

    def __del__(self):
        if self.h:
            self.L.oracle_scene_destroy(self.h)

    def render(self, x_res, y_res, depth, rows=None, threads=1, spp=1, seed=0, cam=None):
        """render.rs:31-38 -> (rgb float32 [y_res, x_res, 3], counters dict).
        rows = (begin, end, step) renders a subset (other rows stay 0).
        spp > 1: jittered supersampling with rt_render_spp's hash (config 5).
        cam: an abi.rt_camera (default Camera::new(x_res, y_res), render.rs:166-176)."""
        from rust_tracer_amd import abi
        cam = cam if cam is not None else abi.camera(x_res, y_res)
        rgb = np.zeros((y_res, x_res, 3), np.float32)
        cnt = (C.c_uint64 * 3)()
        b, e, s = rows if rows is not None else (0, y_res, 1)
        st = self.L.oracle_render_rows_spp_mt(self.h, C.byref(cam), depth, b, e, s, spp, seed,
                                              rgb.ctypes.data_as(C.POINTER(C.c_float)), cnt, threads)
        if st != 0:
            raise RuntimeError(f"oracle_render failed: {st}")
        return rgb, {"node_rays": cnt[0], "shadow_rays": cnt[1], "pixels": cnt[2]}

    def set_material(self, index, material):
        """In-place material edit (desc-built scenes); mirrors rt_scene_set_material."""
        st = self.L.oracle_scene_set_material(self.h, index, C.byref(material))
        if st != 0:
            raise RuntimeError(f"oracle_scene_set_material failed: {st}")

    def forest(self, x_res, y_res, depth, threads=1):
        return OracleForest(self, x_res, y_res, depth, threads)

    def render_forest(self, x_res, y_res, depth):
        from rust_tracer_amd import abi
        cam = abi.camera(x_res, y_res)
        rgb = np.zeros((y_res, x_res, 3), np.float32)
        sizes = np.zeros((y_res, x_res), np.uint32)
        st = self.L.oracle_render_forest(self.h, C.byref(cam), depth,
                                         rgb.ctypes.data_as(C.POINTER(C.c_float)),
                                         sizes.ctypes.data_as(C.POINTER(C.c_uint32)))
        if st != 0:
            raise RuntimeError(f"oracle_render_forest failed: {st}")
        return rgb, sizes


class OracleForest:
    """render_tree.rs RayForest on the CPU (test infrastructure)."""

    def __init__(self, scene, x_res, y_res, depth, threads=1):
        from rust_tracer_amd import abi
        self.L, self.scene = scene.L, scene
        self.w, self.h_res = x_res, y_res
        self.threads = threads
        self.h = C.c_void_p()
        cam = abi.camera(x_res, y_res)
        st = self.L.oracle_forest_build_mt(scene.h, C.byref(cam), depth, threads, C.byref(self.h))
        if st != 0:
            raise RuntimeError(f"oracle_forest_build failed: {st}")

    def __del__(self):
        if getattr(self, "h", None):
            self.L.oracle_forest_destroy(self.h)
            self.h = None

    def render(self):
        rgb = np.zeros((self.h_res, self.w, 3), np.float32)
        self.L.oracle_forest_render_mt(self.h, rgb.ctypes.data_as(C.POINTER(C.c_float)), self.threads)
        return rgb

    def render_filter(self, mutated_ids, rgb):
        rgb = np.array(rgb, np.float32, copy=True)
        ids = (C.c_int32 * max(1, len(mutated_ids)))(*mutated_ids)
        self.L.oracle_forest_render_filter(self.h, ids, len(mutated_ids), rgb.ctypes.data_as(C.POINTER(C.c_float)))
        return rgb

    def tree_sizes(self):
        sizes = np.zeros((self.h_res, self.w), np.uint32)
        self.L.oracle_forest_tree_sizes(self.h, sizes.ctypes.data_as(C.POINTER(C.c_uint32)))
        return sizes

    def trees_with(self, shape_id):
        return int(self.L.oracle_forest_trees_with(self.h, shape_id))


def as_u8(rgb):
    rgb = np.ascontiguousarray(rgb, np.float32)
    out = np.zeros(rgb.shape, np.uint8)
    lib().oracle_as_u8(rgb.ctypes.data_as(C.POINTER(C.c_float)), rgb.size,
                       out.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out


def powf(x, y):
    """libm powf (the reference's f32::powf) elementwise over float32 arrays."""
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y, np.float32)
    out = np.empty_like(x)
    fp = C.POINTER(C.c_float)
    lib().oracle_powf_batch(x.ctypes.data_as(fp), y.ctypes.data_as(fp), out.ctypes.data_as(fp), x.size)
    return out


LIBM_FN = {"powf": 0, "atan2f": 1, "acosf": 2, "atanf": 3}


def libm(fn, x, y=None):
    """The host libm's powf / atan2f(x, y) / acosf / atanf elementwise over float32 arrays
    (the functions the reference's f32 methods call)."""
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y if y is not None else np.zeros_like(x), np.float32)
    out = np.empty_like(x)
    fp = C.POINTER(C.c_float)
    lib().oracle_libm_batch(LIBM_FN[fn], x.ctypes.data_as(fp), y.ctypes.data_as(fp), out.ctypes.data_as(fp), x.size)
    return out
