"""The culling hierarchy (rt_bvh, DESIGN.md "Exact culling") must change nothing.

Every frame rendered with the hierarchy (the default) is compared BIT FOR BIT, with its
ray counters, against the same frame rendered with tuning bvh=0 (every ray tests every
shape, the reference's Scene::intersect loop), and against the CPU oracle where the
oracle finishes in seconds.  The scenes include the adversarial cases of the error
bounds: rays lying in / grazing triangle planes and cube faces, far-away tiny spheres
(large |o'|), anisotropic rotated spheres, reflective planes that launch rays from far
outside the scene, ties (duplicate shapes), glass (rays starting on surfaces).
"""
import os

import numpy as np
import pytest

from oracle.oracle import OracleScene
from rust_tracer_amd import DeviceScene, Matrix, SceneDesc

from .test_gpu_parity import compare

pytestmark = pytest.mark.gpu


def render(desc, w, h, depth, bvh=True):
    s = DeviceScene(desc, tuning=None if bvh else "bvh=0")
    try:
        assert s.uses_bvh == bvh or (bvh and desc.n_shapes == 0)
        s.set_scan_counting(True)
        s.scan_ops(reset=True)
        img, cnt, _, _ = s.render(w, h, depth)
        ops = s.scan_ops()
        return img, cnt, ops
    finally:
        s.close()


def same_both_ways(desc, w, h, depth):
    a, ca, oa = render(desc, w, h, depth, bvh=True)
    b, cb, ob = render(desc, w, h, depth, bvh=False)
    diff = np.flatnonzero(a.view(np.uint32) != b.view(np.uint32))
    assert diff.size == 0, f"{diff.size} values differ, first pixel {np.unravel_index(diff[0] // 3, a.shape[:2])}"
    assert ca == cb
    return a, ca, oa, ob


def test_config3_full_frame_identical():
    """The headline workload: 1920x1080, depth 8, 600 spheres + 25 cubes + 100 triangles."""
    img, cnt, oa, ob = same_both_ways(SceneDesc.synth_config(3), 1920, 1080, 8)
    # the hierarchy must actually cull: far fewer sphere tests than the linear scan
    assert oa["dsph_pairs"] + oa["gsph"] < 0.2 * (ob["dsph_pairs"] + ob["gsph"])
    assert oa["cubes"] < 0.2 * ob["cubes"]


def test_config2_full_frame_identical():
    same_both_ways(SceneDesc.synth_config(2), 1920, 1080, 4)


def test_my_scene_identical():
    same_both_ways(SceneDesc.my_scene(), 640, 480, 8)


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_random_scenes_identical_and_match_oracle(seed):
    desc = SceneDesc.synth(seed, 300, 40, 150, 0.03, 0.6)
    same_both_ways(desc, 320, 180, 8)
    img, cnt, _ = render(desc, 96, 54, 8)
    ref, rcnt = OracleScene(desc).render(96, 54, 8, threads=8)
    compare(img, ref)
    assert cnt == rcnt


def _grazing_scene():
    """Planes of triangles and cube faces that CONTAIN camera rays (camera at z = -8
    looking +z; pixel rows/columns through y = 0 and x = 0 lie in them), triangles a
    hair off those planes, small spheres 50+ units away, anisotropic rotated spheres, a
    mirror floor that sends rays in from far away, duplicate shapes (ties), glass."""
    d = SceneDesc()
    glass = d.phong((0, 0, 0), (1, 1, 1), (1, 1, 1), 60.0, 0.7, 1.5)
    mirror = d.phong((0, 0, 0), (0.3, 0.8, 0.5), (1, 1, 1), 60.0, 0.6, 0.0)
    matte = d.phong((0.05, 0.02, 0.01), (0.5, 0.2, 0.1), (1, 1, 1), 30.0, 0.0, 0.0)
    blue = d.phong((0, 0, 0.1), (0.1, 0.2, 1.0), (1, 1, 1), 80.0, 0.2, 0.0)
    # triangles in the planes y = 0 and x = 0 (contain camera rays) and a hair off them
    d.triangle(matte, (-2, 0, -1), (2, 0, -1), (0, 0, 3))
    d.triangle(blue, (0, -1.5, -2), (0, 1.5, -2), (0, 0, 2))
    d.triangle(mirror, (-2, 1e-6, -1), (2, 1e-6, -1), (0, 1e-6, 3))
    d.triangle(matte, (1e-5, -1, -2), (1e-5, 1, -2), (1e-5, 0, 2))
    d.triangle(blue, (0.5, -0.5, 0), (1.5, -0.5, 0), (1.0, 0.5, 1e-4))
    # axis-aligned cubes whose faces contain camera rays
    d.cube(glass, Matrix.translate(-1.5, 0.5, 0.0))                   # faces at y = 0, y = 1
    d.cube(mirror, Matrix.translate(1.5, -0.5, 1.0) * Matrix.scale(1.0, 1.0, 2.0))
    d.cube(matte, Matrix.translate(0.0, 1.5, 0.5) * Matrix.rotate_y(45.0) * Matrix.scale(0.5, 0.25, 0.5))
    # far small spheres, near-tangent for many pixels
    for k in range(12):
        d.sphere(blue if k % 2 else matte, Matrix.translate(-30 + 5 * k, 0.3 * k - 2, 60.0) * Matrix.scale(0.05, 0.05, 0.05))
    # anisotropic rotated spheres, a duplicate pair, glass
    d.sphere(glass, Matrix.translate(-0.8, -1.0, -2.0) * Matrix.rotate_z(20.0) * Matrix.scale(0.9, 0.3, 0.5))
    d.sphere(mirror, Matrix.translate(0.9, 1.0, -1.0) * Matrix.rotate_x(70.0) * Matrix.scale(0.2, 0.6, 0.3))
    d.sphere(matte, Matrix.translate(0.0, -1.2, 0.5) * Matrix.scale(0.4, 0.4, 0.4))
    d.sphere(blue, Matrix.translate(0.0, -1.2, 0.5) * Matrix.scale(0.4, 0.4, 0.4))
    d.sphere(glass, Matrix.translate(2.2, 1.2, -3.0) * Matrix.scale(0.5, 0.5, 0.5))
    d.plane(mirror, (0.0, -2.0, 0.0), (0.0, 1.0, 0.0))
    d.plane(matte, (0.0, 0.0, 80.0), (0.0, 0.0, -1.0))
    d.point_light((4, 4, 0), (1, 0.9, 0.8))
    d.point_light((-1, 0, -4), (0.3, 1, 0.3))              # in the y = 0 plane
    d.point_light((0, 8, -4), (0.3, 0.3, 1))
    d.set_ambient((0.1, 0.1, 0.1))
    return d


def test_grazing_scene_identical_and_matches_oracle():
    d = _grazing_scene()
    same_both_ways(d, 641, 481, 8)     # odd sizes: the centre row / column are y = 0 / x = 0
    img, cnt, _ = render(d, 161, 121, 8)
    ref, rcnt = OracleScene(d).render(161, 121, 8)
    compare(img, ref)
    assert cnt == rcnt


def test_custom_scene_identical():
    from .test_gpu_parity import _custom_scene
    same_both_ways(_custom_scene(), 320, 240, 12)


def test_counting_kernels_render_the_same_frame():
    """rt_scene_set_scan_counting switches to instrumented kernels; frames must not move."""
    s = DeviceScene(SceneDesc.synth_config(3))
    try:
        a, ca, _, _ = s.render(320, 180, 8)
        s.set_scan_counting(True)
        s.scan_ops(reset=True)
        b, cb, _, _ = s.render(320, 180, 8)
        ops = s.scan_ops()
        s.set_scan_counting(False)
        s.scan_ops(reset=True)
        c, cc, _, _ = s.render(320, 180, 8)
        assert s.scan_ops()["node_pairs"] == 0      # uncounted kernels add nothing
    finally:
        s.close()
    assert ops["node_pairs"] > 0 and ops["dsph_pairs"] > 0
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert np.array_equal(a.view(np.uint32), c.view(np.uint32))
    assert ca == cb == cc


def _render_env(desc, w, h, depth, **tune):
    """One render of a handle created with the given tuning keys (rt_tune.hpp)."""
    s = DeviceScene(desc, tuning=tune or None)
    try:
        img, cnt, _, _ = s.render(w, h, depth)
    finally:
        s.close()
    return img, cnt


def _lights_in_the_cluster():
    """Point lights among the primitives: one inside a glass sphere, one a hair outside a
    matte sphere (no light buffer for them: a grown ball comes within rho of the light),
    one far above (buffered); spheres, cubes and triangles around them."""
    d = SceneDesc.synth(21, 120, 10, 30, 0.05, 0.4).editable()
    glass = d.phong((0, 0, 0), (1, 1, 1), (1, 1, 1), 60.0, 0.7, 1.5)
    matte = d.phong((0.05, 0.05, 0.05), (0.6, 0.5, 0.4), (1, 1, 1), 30.0, 0.0, 0.0)
    d.sphere(glass, Matrix.translate(0.5, 0.2, -0.5) * Matrix.scale(0.6, 0.6, 0.6))
    d.sphere(matte, Matrix.translate(-1.5, 0.8, -1.0) * Matrix.scale(0.3, 0.3, 0.3))
    d.point_light((0.5, 0.2, -0.5), (0.6, 0.6, 0.9))        # inside the glass sphere
    d.point_light((-1.5, 1.11, -1.0), (0.9, 0.5, 0.5))      # 0.01 above the matte sphere
    d.point_light((0.0, 30.0, -4.0), (0.4, 0.4, 0.4))
    return d


@pytest.mark.parametrize("scene", ["config3", "grazing", "lights_in_cluster", "random"])
def test_shadow_shortcuts_change_nothing(scene):
    """Light buffers at several resolutions (lb_res, 0 = off), the trace kernel's own-shape
    shadow tests (self_shadow=0 = off), inline shadow rays (inline_shadow: levels traced
    inline) and the grazing pass's direction cells (graze_res, 0 = cone path): bit-identical
    frames and counters."""
    desc = {"config3": lambda: SceneDesc.synth_config(3), "grazing": _grazing_scene,
            "lights_in_cluster": _lights_in_the_cluster,
            "random": lambda: SceneDesc.synth(31, 400, 30, 120, 0.03, 0.5)}[scene]()
    w, h, depth = 480, 270, 8
    base, cb = _render_env(desc, w, h, depth, lb_res=0, self_shadow=0)
    for env in ({}, {"lb_res": 8}, {"lb_res": 64}, {"lb_res": 200}, {"self_shadow": 0},
                {"inline_shadow": 0}, {"inline_shadow": 8, "lb_res": 16}, {"graze_res": 0},
                {"graze_res": 8}, {"lb_reach": 0}, {"lb_reach": 0, "lb_res": 128},
                {"task_w": 16, "task_fill": 64}):
        img, cnt = _render_env(desc, w, h, depth, **env)
        diff = np.flatnonzero(img.view(np.uint32) != base.view(np.uint32))
        assert diff.size == 0, (env, diff.size)
        assert cnt == cb, env
    if scene == "lights_in_cluster":
        ref, rcnt = OracleScene(desc).render(120, 68, 8, threads=8)
        img, cnt = _render_env(desc, 120, 68, 8)
        compare(img, ref)
        assert cnt == rcnt
