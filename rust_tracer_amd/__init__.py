"""rust_tracer_amd -- MI355X-native render path of erichgess/rust_tracer.

Python face of the C ABI in include/rt_api.h (librt_hip.so, HIP kernels for gfx950).
It mirrors the reference's seam ``render(camera, scene, buffer, depth)``
(src/render.rs:31) and the scene builders of src/my_scene.rs / src/scene.  There is no
CPU render path here: without the built library every call raises.
"""
import ctypes as C
import weakref
import math

import numpy as np

from . import abi
from .abi import (RT_LIGHT_AMBIENT, RT_LIGHT_POINT, RT_MAT_PHONG, RT_MAT_TEXTURE_PHONG,
                  RT_SHAPE_CUBE, RT_SHAPE_PLANE, RT_SHAPE_SPHERE, RT_SHAPE_TRIANGLE,
                  RT_TEX_CHECKERBOARD, RT_TEX_CONST, RtError, camera, check, lib)

__all__ = ["Matrix", "SceneDesc", "DeviceScene", "camera", "render", "RtError", "lib"]

F32 = np.float32
PI_F = F32(math.pi)


class Matrix:
    """Row-major 4x4 f32 (src/math/matrix.rs) with the reference's exact f32 evaluation
    order: products accumulate left to right from 0. (matrix.rs:68-86)."""

    def __init__(self, rows=None):
        self.m = [[F32(0)] * 4 for _ in range(4)] if rows is None else \
            [[F32(v) for v in r] for r in rows]

    @staticmethod
    def identity():
        return Matrix([[1 if i == j else 0 for j in range(4)] for i in range(4)])

    @staticmethod
    def scale(x, y, z):
        m = Matrix.identity()
        m.m[0][0], m.m[1][1], m.m[2][2] = F32(x), F32(y), F32(z)
        return m

    @staticmethod
    def translate(x, y, z):
        m = Matrix.identity()
        m.m[0][3], m.m[1][3], m.m[2][3] = F32(x), F32(y), F32(z)
        return m

    @staticmethod
    def _cs(deg):
        # (angle / 180) * PI in f32; cos/sin evaluated in double then rounded (what
        # rustc's constant folding of rotate_*(const) produces)
        r = F32(F32(deg) / F32(180.0)) * PI_F
        return F32(math.cos(float(r))), F32(math.sin(float(r)))

    @staticmethod
    def rotate_x(deg):
        c, s = Matrix._cs(deg)
        m = Matrix.identity()
        m.m[1][1], m.m[1][2], m.m[2][1], m.m[2][2] = c, -s, s, c
        return m

    @staticmethod
    def rotate_y(deg):
        c, s = Matrix._cs(deg)
        m = Matrix.identity()
        m.m[0][0], m.m[0][2], m.m[2][0], m.m[2][2] = c, s, -s, c
        return m

    @staticmethod
    def rotate_z(deg):
        c, s = Matrix._cs(deg)
        m = Matrix.identity()
        m.m[0][0], m.m[0][1], m.m[1][0], m.m[1][1] = c, -s, s, c
        return m

    def __mul__(self, o):
        r = Matrix()
        for i in range(4):
            for j in range(4):
                acc = F32(0)
                for k in range(4):
                    acc = F32(acc + F32(self.m[i][k] * o.m[k][j]))
                r.m[i][j] = acc
        return r

    def flat(self):
        return [float(v) for row in self.m for v in row]


def _color(c):
    return abi.rt_color(*[float(F32(v)) for v in c])


def phong_material(ambient, diffuse, specular, power, reflectivity, refraction_index):
    """Phong::new (material.rs:33-52) as an rt_material."""
    m = abi.rt_material()
    m.kind = RT_MAT_PHONG
    m.ambient = abi.rt_texture(RT_TEX_CONST, _color(ambient))
    m.diffuse = abi.rt_texture(RT_TEX_CONST, _color(diffuse))
    m.specular = abi.rt_texture(RT_TEX_CONST, _color(specular))
    m.power, m.reflectivity, m.refraction_index = power, reflectivity, refraction_index
    return m


def texture_phong_material(ambient, diffuse, specular, power, reflectivity, refraction_index):
    """TexturePhong::new (material.rs:112-131); a texture is an RGB tuple or 'checkerboard'."""
    def tex(t):
        if isinstance(t, str):
            assert t == "checkerboard"
            return abi.rt_texture(RT_TEX_CHECKERBOARD, abi.rt_color(0, 0, 0))
        return abi.rt_texture(RT_TEX_CONST, _color(t))
    m = abi.rt_material()
    m.kind = RT_MAT_TEXTURE_PHONG
    m.ambient, m.diffuse, m.specular = tex(ambient), tex(diffuse), tex(specular)
    m.power, m.reflectivity, m.refraction_index = power, reflectivity, refraction_index
    return m


class SceneDesc:
    """An rt_scene_desc: either produced by the C++ host builders (my_scene, synth,
    bench_128) or assembled here shape by shape (Scene::add_shape order)."""

    def __init__(self):
        self._owned_ptr = None      # pointer from an rt_desc_* builder
        self.materials, self.shapes, self.lights = [], [], []
        self.ambient = (0.0, 0.0, 0.0)
        self._keep = None

    # ---- builders in librt_hip.so
    @classmethod
    def _from_builder(cls, fn, *args):
        d = cls()
        p = C.POINTER(abi.rt_scene_desc)()
        check(fn(*args, C.byref(p)), fn.__name__)
        d._owned_ptr = p
        return d

    @classmethod
    def my_scene(cls):
        """src/my_scene.rs:45-120"""
        return cls._from_builder(lib().rt_desc_my_scene)

    @classmethod
    def bench_128(cls):
        """src/render.rs:233-249"""
        return cls._from_builder(lib().rt_desc_bench_128)

    @classmethod
    def synth(cls, seed, n_spheres, n_cubes=0, n_triangles=0, r_min=0.06, r_max=0.2):
        p = abi.rt_synth_params(seed, n_spheres, n_cubes, n_triangles, r_min, r_max)
        return cls._from_builder(lib().rt_desc_synth, C.byref(p))

    @classmethod
    def synth_config(cls, config):
        """BASELINE.json configs 2..5."""
        p = abi.rt_synth_params()
        check(lib().rt_synth_config(config, C.byref(p)), "rt_synth_config")
        return cls._from_builder(lib().rt_desc_synth, C.byref(p))

    def editable(self):
        """A Python-assembled copy (shapes / lights / materials can be appended)."""
        d = SceneDesc()
        src = self.ptr().contents
        d.materials = [abi.rt_material.from_buffer_copy(src.materials[i]) for i in range(src.n_materials)]
        d.shapes = [abi.rt_shape.from_buffer_copy(src.shapes[i]) for i in range(src.n_shapes)]
        d.lights = [abi.rt_light.from_buffer_copy(src.lights[i]) for i in range(src.n_lights)]
        d.ambient = (src.ambient.r, src.ambient.g, src.ambient.b)
        return d

    # ---- assembled in Python
    def phong(self, ambient, diffuse, specular, power, reflectivity, refraction_index):
        self.materials.append(phong_material(ambient, diffuse, specular, power, reflectivity,
                                             refraction_index))
        return len(self.materials) - 1

    def texture_phong(self, ambient, diffuse, specular, power, reflectivity, refraction_index):
        """Each texture is an RGB tuple (constant) or the string 'checkerboard'."""
        self.materials.append(texture_phong_material(ambient, diffuse, specular, power, reflectivity,
                                                     refraction_index))
        return len(self.materials) - 1

    def _shape(self, kind, mat, transform=None, data=()):
        s = abi.rt_shape()
        s.kind, s.material = kind, mat
        s.transform[:] = (transform or Matrix.identity()).flat()
        for i, v in enumerate(data):
            s.data[i] = float(F32(v))
        self.shapes.append(s)
        return len(self.shapes) - 1

    def sphere(self, mat, transform=None):
        return self._shape(RT_SHAPE_SPHERE, mat, transform)

    def plane(self, mat, origin, normal, transform=None):
        return self._shape(RT_SHAPE_PLANE, mat, transform, tuple(origin) + tuple(normal))

    def triangle(self, mat, v0, v1, v2):
        return self._shape(RT_SHAPE_TRIANGLE, mat, None, tuple(v0) + tuple(v1) + tuple(v2))

    def cube(self, mat, transform=None):
        return self._shape(RT_SHAPE_CUBE, mat, transform)

    def point_light(self, pos, color):
        l = abi.rt_light()
        l.kind = RT_LIGHT_POINT
        l.pos[:] = [float(F32(v)) for v in pos]
        l.color = _color(color)
        self.lights.append(l)

    def ambient_light(self, color):
        l = abi.rt_light()
        l.kind = RT_LIGHT_AMBIENT
        l.color = _color(color)
        self.lights.append(l)

    def set_ambient(self, color):
        self.ambient = color

    def ptr(self):
        """POINTER(rt_scene_desc) valid while this object lives."""
        if self._owned_ptr is not None:
            return self._owned_ptr
        mats = (abi.rt_material * max(1, len(self.materials)))(*self.materials)
        shapes = (abi.rt_shape * max(1, len(self.shapes)))(*self.shapes)
        lights = (abi.rt_light * max(1, len(self.lights)))(*self.lights)
        d = abi.rt_scene_desc(len(self.materials), mats, len(self.shapes), shapes,
                              len(self.lights), lights, _color(self.ambient))
        self._keep = (mats, shapes, lights, d)
        return C.pointer(d)

    @property
    def n_shapes(self):
        return self.ptr().contents.n_shapes

    def __del__(self):
        if self._owned_ptr is not None and abi._lib is not None:
            abi._lib.rt_desc_free(self._owned_ptr)
            self._owned_ptr = None


def tuning_spec(tuning):
    """bytes for the C ABI from None, "k=v,..." or {k: v}."""
    if tuning is None:
        return None
    if isinstance(tuning, dict):
        tuning = ",".join(f"{k}={v}" for k, v in tuning.items())
    return tuning.encode()


class DeviceScene:
    """An uploaded scene (rt_scene_create) on one HIP device, or -- `devices` a list --
    replicated over several (rt_scene_create_multi: render() then tiles the frame across
    them and gathers it over RCCL, from this one thread)."""

    def __init__(self, desc, device=-1, devices=None, tuning=None, _handle=None):
        """tuning: "key=value,..." of rust_tracer_amd/csrc/rt_tune.hpp (rt_scene_create_tuned;
        every key is exact -- it moves time, never a pixel), or a dict of them."""
        self._L = lib()
        self.h = C.c_void_p()
        self.desc = desc
        if _handle is not None:
            self.h = _handle
        elif devices is not None:
            assert tuning is None, "multi-device scenes take their tuning from RT_TUNE"
            arr = (C.c_int32 * len(devices))(*devices)
            check(self._L.rt_scene_create_multi(desc.ptr(), arr, len(devices), C.byref(self.h)),
                  "rt_scene_create_multi")
        else:
            check(self._L.rt_scene_create_tuned(desc.ptr(), device, tuning_spec(tuning), C.byref(self.h)),
                  "rt_scene_create_tuned")

    def set_tuning(self, tuning):
        """rt_scene_set_tuning: change per-pass keys of rt_tune.hpp (string or dict)."""
        check(self._L.rt_scene_set_tuning(self.h, tuning_spec(tuning)), "rt_scene_set_tuning")

    def clone(self, device=-1):
        """rt_scene_clone: another handle of this scene (own workspace and stream), copied on
        the device without rebuilding it."""
        h = C.c_void_p()
        check(self._L.rt_scene_clone(self.h, device, C.byref(h)), "rt_scene_clone")
        return DeviceScene(self.desc, _handle=h)

    @property
    def device_count(self):
        return int(self._L.rt_scene_device_count(self.h))

    @property
    def uses_rccl(self):
        return bool(self._L.rt_scene_uses_rccl(self.h))

    def sync_status(self):
        """rt_scene_sync_status: wait for this scene's stream-ordered renders; raises
        RtError(RT_ERR_CAPACITY) if one of them overflowed a ray queue (incomplete frame)."""
        check(self._L.rt_scene_sync_status(self.h), "rt_scene_sync_status")

    def close(self):
        if self.h:
            # forests of this scene first: rt_forest_destroy uses its scene's stream.  (A cycle
            # holding both -- e.g. a test frame kept by a traceback -- is finalised in any order)
            for f in list(getattr(self, "_forests", ())):
                f.close()
            self._L.rt_scene_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def flops_per_scan(self):
        return int(self._L.rt_scene_flops_per_scan(self.h))

    @property
    def device_bytes(self):
        return int(self._L.rt_scene_device_bytes(self.h))

    @property
    def workspace_bytes(self):
        """rt_scene_workspace_bytes: device bytes of this handle's render workspace."""
        return int(self._L.rt_scene_workspace_bytes(self.h))

    @property
    def uses_bvh(self):
        """True when scans walk the culling hierarchy (RT_BVH=0 at creation turns it off)."""
        return bool(self._L.rt_scene_uses_bvh(self.h))

    SCAN_OPS = ("node_pairs", "dsph_pairs", "gsph", "tri_pairs", "cube_boxes", "cubes", "graze_cones",
                "planes", "graze_normals", "cycles_nodes", "cycles_leaves", "cycles_graze", "cycles_scans",
                "cycles_load", "cycles_post", "cycles_self")

    def set_grid_share(self, percent):
        """rt_scene_set_grid_share: persistent grids at `percent` % of a full chip (frames in
        flight: several passes side by side)."""
        check(self._L.rt_scene_set_grid_share(self.h, int(percent)), "rt_scene_set_grid_share")
        self._grid_share = int(percent)

    @property
    def grid_share(self):
        """The share set by set_grid_share (100 = a full chip, the default of a new handle)."""
        return getattr(self, "_grid_share", 100)

    def set_scan_counting(self, enable=True):
        """Run the instrumented (counting) kernels from now on (rt_scene_set_scan_counting)."""
        check(self._L.rt_scene_set_scan_counting(self.h, 1 if enable else 0), "rt_scene_set_scan_counting")

    def scan_ops(self, reset=False):
        """Lane-weighted test counts since the last reset (rt_scene_scan_ops)."""
        out = (C.c_uint64 * len(self.SCAN_OPS))()
        check(self._L.rt_scene_scan_ops(self.h, out, len(self.SCAN_OPS), 1 if reset else 0),
              "rt_scene_scan_ops")
        return dict(zip(self.SCAN_OPS, (int(v) for v in out)))

    def render(self, x_res, y_res, depth, want_u8=False, device=-1, spp=1, seed=0, cam=None, out=None):
        """render.rs:31-38 -> (rgb float32 [y_res, x_res, 3], counters dict, kernel_ms, rgb8).
        spp > 1: jittered supersampling (rt_render_spp, BASELINE config 5).  cam: an
        abi.rt_camera (default Camera::new(x_res, y_res), render.rs:166-176).  out: the
        caller's float32 [y_res, x_res, 3] buffer to fill (e.g. a HostFrame's array)."""
        cam = cam if cam is not None else camera(x_res, y_res)
        if out is not None:
            assert out.dtype == np.float32 and out.shape == (y_res, x_res, 3) and out.flags.c_contiguous
        rgb = out if out is not None else np.zeros((y_res, x_res, 3), np.float32)
        rgb8 = np.zeros((y_res, x_res, 3), np.uint8) if want_u8 else None
        cnt = abi.rt_counters()
        ms = C.c_float(0)
        opts = abi.rt_render_opts(device, C.pointer(cnt), C.pointer(ms))
        check(self._L.rt_render_spp(self.h, C.byref(cam), depth, spp, seed, C.byref(opts),
                                    rgb.ctypes.data_as(C.POINTER(C.c_float)),
                                    rgb8.ctypes.data_as(C.POINTER(C.c_uint8)) if want_u8 else None),
              "rt_render_spp")
        counters = {"node_rays": cnt.node_rays, "shadow_rays": cnt.shadow_rays,
                    "pixels": cnt.pixels}
        self.last_wave_iterations = cnt.wave_iterations
        return rgb, counters, ms.value, rgb8

    KERNEL_KINDS = ("trace", "sort_tasks", "sort_shadow", "shadow", "combine")

    def set_kernel_timing(self, enable=True):
        """rt_scene_set_kernel_timing: bracket every launch group of this handle's passes with
        HIP events (measurement only)."""
        check(self._L.rt_scene_set_kernel_timing(self.h, 1 if enable else 0), "rt_scene_set_kernel_timing")

    def kernel_times(self, reset=False):
        """rt_scene_kernel_times: ms per kernel kind summed over the timed passes, and the
        number of launch groups timed."""
        out = (C.c_float * (len(self.KERNEL_KINDS) + 1))()
        check(self._L.rt_scene_kernel_times(self.h, out, len(out), 1 if reset else 0), "rt_scene_kernel_times")
        d = dict(zip(self.KERNEL_KINDS, (float(v) for v in out)))
        d["launch_groups"] = int(out[len(self.KERNEL_KINDS)])
        return d

    def set_material(self, index, material):
        """rt_scene_set_material: replace material `index` (same kind), e.g. the GUI's edits."""
        check(self._L.rt_scene_set_material(self.h, index, C.byref(material)), "rt_scene_set_material")

    UPDATE_KINDS = {0: "unchanged", 1: "materials", 2: "rebuilt"}

    def update(self, desc):
        """rt_scene_update: bring this handle up to date with `desc` (the caller's scene after
        edits) -- nothing when unchanged, material edits in place, else a rebuild adopted by
        this handle.  Returns "unchanged" / "materials" / "rebuilt"."""
        what = C.c_int32(0)
        check(self._L.rt_scene_update(self.h, desc.ptr(), C.byref(what)), "rt_scene_update")
        self.desc = desc
        return self.UPDATE_KINDS[what.value]

    def forest(self, x_res, y_res, depth):
        """generate_ray_forest (render_tree.rs:147-164) on the device."""
        return DeviceForest(self, x_res, y_res, depth)

    def render_bands_async(self, cam, depth, band_rows, rank, world, d_rgb_ptr, d_counters_ptr,
                           stream_ptr, spp=1, seed=0):
        check(self._L.rt_render_bands_spp_async(self.h, C.byref(cam), depth, spp, seed, band_rows, rank, world,
                                                C.c_void_p(d_rgb_ptr), C.c_void_p(d_counters_ptr),
                                                C.c_void_p(stream_ptr)), "rt_render_bands_spp_async")

    def render_frame_async(self, cam, depth, d_rgb_ptr, d_counters_ptr, stream_ptr, d_rgb8_ptr=0):
        """rt_render_frame_async: the whole frame, row-major, into device memory on `stream_ptr`
        (rt_render's two band shares side by side, forked from and joined into that stream)."""
        check(self._L.rt_render_frame_async(self.h, C.byref(cam), depth, C.c_void_p(d_rgb_ptr),
                                             C.c_void_p(d_rgb8_ptr or None), C.c_void_p(d_counters_ptr or None),
                                             C.c_void_p(stream_ptr)), "rt_render_frame_async")

    def render_bands_ex_async(self, cams, depth, band_rows, rank, world, d_rgb_ptr, d_rgb8_ptr, d_counters_ptr,
                              stream_ptr, spp=1, seed=0):
        """rt_render_bands_ex_async: len(cams) frames; f32 bands (d_rgb_ptr, may be 0 when
        spp == 1 and d_rgb8_ptr is given) and / or fused RGB8 bands (d_rgb8_ptr)."""
        arr = (abi.rt_camera * len(cams))(*cams)
        check(self._L.rt_render_bands_ex_async(self.h, arr, len(cams), depth, spp, seed, band_rows, rank, world,
                                               C.c_void_p(d_rgb_ptr or None), C.c_void_p(d_rgb8_ptr or None),
                                               C.c_void_p(d_counters_ptr or None), C.c_void_p(stream_ptr)),
              "rt_render_bands_ex_async")

    def render_bands_direct_async(self, cams, depth, band_rows, rank, world, d_frames_ptr, d_frames8_ptr,
                                  d_counters_ptr, stream_ptr):
        """rt_render_bands_direct_async: this rank's rows of len(cams) whole row-major frames,
        written in place (f32 at d_frames_ptr and / or RGB8 at d_frames8_ptr)."""
        arr = (abi.rt_camera * len(cams))(*cams)
        check(self._L.rt_render_bands_direct_async(self.h, arr, len(cams), depth, band_rows, rank, world,
                                                   C.c_void_p(d_frames_ptr or None), C.c_void_p(d_frames8_ptr or None),
                                                   C.c_void_p(d_counters_ptr or None), C.c_void_p(stream_ptr)),
              "rt_render_bands_direct_async")

    def render_bands_batch_async(self, cams, depth, band_rows, rank, world, d_rgb_ptr, d_counters_ptr, stream_ptr):
        """rt_render_bands_batch_async: len(cams) frames (<= rt_max_frames() = 32, one resolution) in one pipeline
        pass into len(cams) consecutive band buffers."""
        arr = (abi.rt_camera * len(cams))(*cams)
        check(self._L.rt_render_bands_batch_async(self.h, arr, len(cams), depth, band_rows, rank, world,
                                                  C.c_void_p(d_rgb_ptr), C.c_void_p(d_counters_ptr),
                                                  C.c_void_p(stream_ptr)), "rt_render_bands_batch_async")


class DeviceForest:
    """A RayForest kept on the device (rt_forest_*): built once, shaded any number of times."""

    def __init__(self, scene, x_res, y_res, depth):
        self._L = lib()
        self.scene = scene  # keeps the scene alive
        self.w, self.h_res = x_res, y_res
        self.h = C.c_void_p()
        cam = camera(x_res, y_res)
        check(self._L.rt_forest_create(scene.h, C.byref(cam), depth, C.byref(self.h)), "rt_forest_create")
        if not hasattr(scene, "_forests"):
            scene._forests = weakref.WeakSet()
        scene._forests.add(self)

    def close(self):
        if self.h:
            self._L.rt_forest_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def render(self):
        """render_forest (render_tree.rs:121-127) -> rgb float32 [y, x, 3]"""
        rgb = np.zeros((self.h_res, self.w, 3), np.float32)
        check(self._L.rt_forest_render(self.h, rgb.ctypes.data_as(C.POINTER(C.c_float))), "rt_forest_render")
        return rgb

    def render_filter(self, mutated_ids, rgb):
        """render_forest_filter (render_tree.rs:129-145): a copy of `rgb` in which the pixels
        whose tree holds a mutated shape id are re-shaded (the others keep their values)."""
        rgb = np.array(rgb, np.float32, order="C", copy=True)
        ids = (C.c_int32 * max(1, len(mutated_ids)))(*mutated_ids)
        check(self._L.rt_forest_render_filter(self.h, ids, len(mutated_ids),
                                              rgb.ctypes.data_as(C.POINTER(C.c_float))),
              "rt_forest_render_filter")
        return rgb

    def tree_sizes(self):
        sizes = np.zeros((self.h_res, self.w), np.uint32)
        check(self._L.rt_forest_tree_sizes(self.h, sizes.ctypes.data_as(C.POINTER(C.c_uint32))),
              "rt_forest_tree_sizes")
        return sizes

    def trees_with(self, shape_id):
        n = C.c_uint64(0)
        check(self._L.rt_forest_trees_with(self.h, shape_id, C.byref(n)), "rt_forest_trees_with")
        return int(n.value)

    def counters(self):
        c = abi.rt_counters()
        check(self._L.rt_forest_counters(self.h, C.byref(c)), "rt_forest_counters")
        return {"node_rays": c.node_rays, "shadow_rays": c.shadow_rays, "pixels": c.pixels}

    def timings(self):
        """rt_forest_timings: device ms of the build's trace + shadow passes and of the last
        render / render_filter (mark + shade kernels, host copies excluded)."""
        b, sh = C.c_float(0), C.c_float(0)
        check(self._L.rt_forest_timings(self.h, C.byref(b), C.byref(sh)), "rt_forest_timings")
        return {"build_ms": b.value, "shade_ms": sh.value}

    def stats(self):
        """RayForest::stats (render_tree.rs:73-93), including its f32 percentile indexing."""
        sizes = np.sort(self.tree_sizes().ravel(order="F"))  # the reference iterates forest[u][v]
        n = len(sizes)

        def at(q):
            return int(sizes[int(np.float32(q) * np.float32(n))])
        return {"num_trees": n, "num_intersections": int(sizes.sum()), "smallest_tree": int(sizes.min()),
                "largest_tree": int(sizes.max()), "median": int(sizes[n // 2]), "p90": at(0.9),
                "p95": at(0.95), "p99": at(0.99)}


class _PinnedBuffer:
    """rt_host_alloc'd bytes exposed through the array interface: every numpy view of it keeps
    this object (and so the page-locked allocation) alive; the last view to go frees it."""

    def __init__(self, nbytes):
        self._L = lib()
        self.ptr = C.c_void_p()
        check(self._L.rt_host_alloc(nbytes, C.byref(self.ptr)), "rt_host_alloc")
        self.__array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (self.ptr.value, False),
                                    "version": 3}

    def __del__(self):
        try:
            if self.ptr:
                self._L.rt_host_free(self.ptr)
                self.ptr = C.c_void_p()
        except Exception:
            pass


class HostFrame:
    """A float32 [h, w, 3] frame in page-locked host memory (rt_host_alloc): rt_render's
    device-to-host copy into it runs at the link's DMA rate.  The allocation lives as long as
    any array view of it (``HostFrame(w, h).array`` alone is safe); close() drops this
    object's own reference."""

    def __init__(self, w, h):
        self.array = np.asarray(_PinnedBuffer(w * h * 3 * 4)).view(np.float32).reshape(h, w, 3)

    def close(self):
        self.array = None


def write_image(path, rgb8):
    """rt_write_image: save an RGB8 frame [y, x, 3] as .png / .bmp / .ppm (host code)."""
    rgb8 = np.ascontiguousarray(rgb8, np.uint8)
    check(lib().rt_write_image(str(path).encode(), rgb8.ctypes.data_as(C.POINTER(C.c_uint8)),
                               rgb8.shape[1], rgb8.shape[0]), "rt_write_image")


def band_rows_per_rank(y_res, band_rows, world):
    return int(lib().rt_band_rows_per_rank(y_res, band_rows, world))


def unpermute_bands_async(d_gathered_ptr, x_res, y_res, band_rows, world, d_frame_ptr, stream_ptr):
    check(lib().rt_unpermute_bands_async(C.c_void_p(d_gathered_ptr), x_res, y_res, band_rows, world,
                                         C.c_void_p(d_frame_ptr), C.c_void_p(stream_ptr)),
          "rt_unpermute_bands_async")


def unpermute_bands_u8_async(d_gathered_ptr, x_res, y_res, band_rows, world, d_frame_ptr, stream_ptr):
    check(lib().rt_unpermute_bands_u8_async(C.c_void_p(d_gathered_ptr), x_res, y_res, band_rows, world,
                                            C.c_void_p(d_frame_ptr), C.c_void_p(stream_ptr)),
          "rt_unpermute_bands_u8_async")


def unpermute_bands_batch_async(d_gathered_ptr, x_res, y_res, band_rows, world, n_frames, stride_frames,
                                d_frames_ptr, stream_ptr, rgb8=False):
    """rt_unpermute_bands_batch_async (_u8 with rgb8): n_frames frames of one gather of every
    rank's batch band buffers (stride_frames buffers per rank) into consecutive frames."""
    f = lib().rt_unpermute_bands_batch_u8_async if rgb8 else lib().rt_unpermute_bands_batch_async
    check(f(C.c_void_p(d_gathered_ptr), x_res, y_res, band_rows, world, n_frames, stride_frames,
            C.c_void_p(d_frames_ptr), C.c_void_p(stream_ptr)), "rt_unpermute_bands_batch_async")


def quantize_u8_async(d_rgb_ptr, n, d_rgb8_ptr, stream_ptr):
    check(lib().rt_quantize_u8_async(C.c_void_p(d_rgb_ptr), n, C.c_void_p(d_rgb8_ptr),
                                     C.c_void_p(stream_ptr)), "rt_quantize_u8_async")


def render(x_res, y_res, desc, depth, device=-1, want_u8=False):
    """One-shot: upload `desc`, render, release (the reference's render() seam)."""
    s = DeviceScene(desc, device)
    try:
        return s.render(x_res, y_res, depth, want_u8=want_u8, device=device)
    finally:
        s.close()


def mirror_render_calls(scene, x_res, y_res, depth, n_calls, edit=0, device=-1, fresh=False):
    """rt_mirror_render_calls (include/rt_scenes.h): the C++ mirror's render() called n_calls
    times on one Scene (the reference's bench loop through the drop-in seam).  scene: 0 =
    my_scene, 2..5 = BASELINE configs; edit before the last call: 0 none, 1 set_transform,
    2 material, 3 light.  Returns (ms per call, update kinds per call, last frame, the frame of a
    fresh handle of the edited scene or None)."""
    L = lib()
    ms = (C.c_float * n_calls)()
    up = (C.c_int32 * n_calls)()
    rgb = np.zeros((y_res, x_res, 3), np.float32)
    ref = np.zeros((y_res, x_res, 3), np.float32) if fresh else None
    fp = C.POINTER(C.c_float)
    check(L.rt_mirror_render_calls(scene, x_res, y_res, depth, n_calls, edit, device, ms, up,
                                   rgb.ctypes.data_as(fp), ref.ctypes.data_as(fp) if fresh else None),
          "rt_mirror_render_calls")
    return list(ms), list(up), rgb, ref
