"""Exactness of the culling hierarchy outside the benchmark scenes.

The hierarchy walk, the grazing pass and the light buffers skip primitives only when
bounds (DESIGN.md "Why skipping is exact") prove no hit the reference could report is
lost; Scene::intersect (src/scene/mod.rs:98-116) tests every shape.  These scenes push the
bounds where the benchmark scenes do not: world scales x0.01 / x100 / x1000 (with the
reference's absolute 0.0002 offsets and absolute light-buffer radii), cameras far from the
scene and inside it, point lights within 0.05 of a primitive (no light buffer), sliver
triangles (sin(angle) ~ 1e-3, linear-scan candidates), anisotropic rotated spheres,
duplicate shapes.  Each is rendered with the hierarchy and with tuning bvh=0 (every shape
tested for every ray): frames and ray counters must be identical bit for bit; and at a
small size against the CPU oracle.
"""
import numpy as np
import pytest

from oracle.oracle import OracleScene
from rust_tracer_amd import DeviceScene, Matrix, SceneDesc, abi

pytestmark = pytest.mark.gpu


def stress_scene(seed, scale, near_lights, slivers):
    rng = np.random.default_rng(seed)
    s = float(scale)
    d = SceneDesc()
    mats = [d.phong((0.02, 0.02, 0.02), tuple(rng.uniform(0.2, 1.0, 3)), (1, 1, 1), 60.0, 0.0, 0.0),
            d.phong((0, 0, 0), tuple(rng.uniform(0.2, 1.0, 3)), (1, 1, 1), 60.0, 0.5, 0.0),
            d.phong((0, 0, 0), (1, 1, 1), (1, 1, 1), 60.0, 0.7, 1.333),
            d.texture_phong((0.05, 0.05, 0.05), "checkerboard", (1, 1, 1), 600.0, 0.2, 0.0)]
    d.plane(mats[3], (0.0, -2.0 * s, 0.0), (0.0, 1.0, 0.0))
    d.plane(mats[3], (0.0, 0.0, 6.0 * s), (0.0, 0.0, -1.0), Matrix.rotate_y(10.0))
    lo, hi = np.array([-3.0, -1.9, -3.0]) * s, np.array([3.0, 2.5, 1.5]) * s
    spheres = []
    for i in range(140):
        c = rng.uniform(lo, hi)
        r = float(rng.uniform(0.03, 0.5)) * s
        m = mats[int(rng.integers(0, 3))]
        if rng.random() < 0.15:
            t = Matrix.translate(*c) * Matrix.rotate_z(float(rng.uniform(0, 90))) * Matrix.scale(r, 0.3 * r, r)
        else:
            t = Matrix.translate(*c) * Matrix.scale(r, r, r)
        d.sphere(m, t)
        spheres.append((c, r))
    d.sphere(mats[0], Matrix.translate(*spheres[3][0]) * Matrix.scale(spheres[3][1], spheres[3][1], spheres[3][1]))
    for i in range(18):
        c = rng.uniform(lo, hi)
        k = float(rng.uniform(0.1, 0.6)) * s
        t = (Matrix.translate(*c) * Matrix.rotate_x(float(rng.uniform(-60, 60))) *
             Matrix.rotate_y(float(rng.uniform(0, 90))) * Matrix.scale(k, k, k))
        d.cube(mats[int(rng.integers(0, 3))], t)
    for i in range(60):
        v0 = rng.uniform(lo, hi)
        v1 = v0 + rng.uniform(-0.4, 0.4, 3) * s
        v2 = v0 + rng.uniform(-0.4, 0.4, 3) * s
        d.triangle(mats[int(rng.integers(0, 4))], v0, v1, v2)
    if slivers:
        for i in range(20):
            v0 = rng.uniform(lo, hi)
            e = rng.uniform(-0.6, 0.6, 3) * s
            nrm = np.cross(e, rng.normal(size=3))
            nrm /= np.linalg.norm(nrm)
            v2 = v0 + float(rng.uniform(0.2, 0.8)) * e + nrm * float(rng.uniform(1e-4, 2e-3)) * np.linalg.norm(e)
            d.triangle(mats[int(rng.integers(0, 3))], v0, v0 + e, v2)
    d.point_light((-4.0 * s, 5.0 * s, -6.0 * s), (0.8, 0.8, 0.8))
    d.point_light((3.0 * s, 3.5 * s, -2.0 * s), (0.6, 0.5, 0.4))
    if near_lights:  # within 0.02 (scaled) of a sphere's surface, and one just off a triangle
        c, r = spheres[7]
        u = rng.normal(size=3)
        u /= np.linalg.norm(u)
        d.point_light(tuple(c + u * (r + 0.02 * s)), (0.7, 0.7, 0.9))
    else:
        d.point_light((0.5 * s, 4.0 * s, -1.0 * s), (0.5, 0.5, 0.5))
    d.set_ambient((0.1, 0.1, 0.1))
    d.stress_spheres = spheres  # (centre, radius) of the axis-aligned ones' balls
    return d


def stress_camera(w, h, scale, mode):
    """Camera::new's window [-3, 3]^2 at z = 0, scaled; the origin (0, 0, -8) scaled, far
    away (z = -800), or inside the cloud of shapes."""
    cam = abi.camera(w, h)
    s = float(scale)
    origin = {"std": (0.0, 0.0, -8.0), "far": (0.0, 0.4, -800.0), "inside": (0.3, 0.2, -1.0)}[mode]
    cam.origin[:] = tuple(float(np.float32(v * s)) for v in origin)
    cam.x_min, cam.x_max = float(np.float32(-3.0 * s)), float(np.float32(3.0 * s))
    cam.y_min, cam.y_max = float(np.float32(-3.0 * s)), float(np.float32(3.0 * s))
    return cam


CASES = [
    # seed, scale, camera, near lights, slivers
    (21, 0.01, "std", False, False),
    (22, 0.01, "far", True, True),
    (23, 100.0, "std", True, False),
    (24, 100.0, "far", False, True),
    (25, 1.0, "inside", True, True),
    (26, 1.0, "far", True, True),
    (27, 1000.0, "std", True, True),
    (28, 0.01, "inside", True, True),
]


def same_bits(a, b):
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("seed,scale,cam_mode,near,slivers", CASES)
def test_hierarchy_is_exact_under_stress(seed, scale, cam_mode, near, slivers, monkeypatch):
    desc = stress_scene(seed, scale, near, slivers)
    w, h, depth = 160, 120, 6
    cam = stress_camera(w, h, scale, cam_mode)
    s = DeviceScene(desc, device=0)
    assert s.uses_bvh
    img, cnt, _, _ = s.render(w, h, depth, cam=cam)
    s.close()
    s = DeviceScene(desc, device=0, tuning="bvh=0")
    assert not s.uses_bvh
    ref, rcnt, _, _ = s.render(w, h, depth, cam=cam)
    s.close()
    assert cnt == rcnt
    mism = ~(img.view(np.uint32) == ref.view(np.uint32)).all(axis=2)
    assert not mism.any(), f"{int(mism.sum())} pixels differ, first at {np.argwhere(mism)[:5].tolist()}"
    assert cnt["node_rays"] > w * h // 4  # the scene is in view


@pytest.mark.parametrize("seed,scale,cam_mode,near,slivers", CASES)
def test_stress_scenes_match_oracle(seed, scale, cam_mode, near, slivers):
    """Every stress scene at the hierarchy test's size (160x120, depth 6) against the oracle:
    the culling hierarchy, light-buffer tiers, shape buffers and grazing pass together."""
    desc = stress_scene(seed, scale, near, slivers)
    w, h, depth = 160, 120, 6
    cam = stress_camera(w, h, scale, cam_mode)
    s = DeviceScene(desc, device=0)
    img, cnt, _, _ = s.render(w, h, depth, cam=cam)
    s.close()
    ref, rcnt = OracleScene(desc).render(w, h, depth, cam=cam, threads=8)
    assert cnt == rcnt
    diff = np.abs(img.astype(np.float64) - ref.astype(np.float64))
    both_nan = np.isnan(img) & np.isnan(ref)
    diff[both_nan] = 0.0
    assert not np.isnan(diff).any()
    assert float(diff.max()) <= 1e-4  # north_star: every RGB channel within 1e-4
    differ = ~((img.view(np.uint32) == ref.view(np.uint32)) | both_nan)
    print(f"stress {seed}: max |diff| {float(diff.max()):.3g}, channels differing {int(differ.sum())}")


@pytest.mark.parametrize("case", [None] + CASES[:3] + CASES[4:5])
def test_shape_buffers_change_nothing(case, monkeypatch):
    """Rays inside a sphere test its shape buffer instead of walking the hierarchy (rt_build.cpp
    build_shape_buffers): frames and counters identical to the walk (RT_SHAPE_BUF=0) and to
    the key mode without inside rays (task_key=6)."""
    if case is None:
        desc, w, h, depth, cam = SceneDesc.synth_config(3), 480, 270, 8, None
    else:
        seed, scale, cam_mode, near, slivers = case
        desc, w, h, depth = stress_scene(seed, scale, near, slivers), 160, 120, 8
        cam = stress_camera(w, h, scale, cam_mode)
    out = []
    for tune in (None, "shape_buf=0", "task_key=6"):
        s = DeviceScene(desc, device=0, tuning=tune)
        out.append(s.render(w, h, depth, cam=cam)[:2])
        s.close()
    for img, cnt in out[1:]:
        assert same_bits(img, out[0][0]) and cnt == out[0][1]


@pytest.mark.parametrize("case", [None] + CASES)
def test_light_buffer_tiers_change_nothing(case):
    """Light-buffer tiers (rt_build.cpp build_light_buffers: tier t serves shadow-ray origins
    with D <= 3 R 2^t and a light within 45 * 2^t, its records' balls grown by their bound at
    that reach): frames and counters identical with one tier, the default, seven, no light
    buffers at all (every shadow ray walks the hierarchy), and six tiers for every light with
    the records near the light in every cell of a tier (lb_near_all)."""
    if case is None:
        desc, w, h, depth, cam = SceneDesc.synth_config(3), 480, 270, 8, None
    else:
        seed, scale, cam_mode, near, slivers = case
        desc, w, h, depth = stress_scene(seed, scale, near, slivers), 160, 120, 8
        cam = stress_camera(w, h, scale, cam_mode)
    out = []
    for tune in (None, "lb_tiers=1", "lb_tiers=7", "lb_res=0", "lb_near_all=1,lb_tiers=6"):
        s = DeviceScene(desc, device=0, tuning=tune)
        out.append(s.render(w, h, depth, cam=cam)[:2])
        s.close()
    for img, cnt in out[1:]:
        assert same_bits(img, out[0][0]) and cnt == out[0][1]


@pytest.mark.parametrize("case", [None] + CASES)
def test_far_shadow_walks_change_nothing(case):
    """Shadow waves whose walk cannot cull (the box growth h(D) of their nearest walking origin
    spans walk_linear scene radii: the far floor) test every hierarchy primitive linearly
    (rt_scan.hpp hier_linear), and the walking rays sort first in the shadow queue
    (walk_first): frames and counters identical to the walk for every wave, to the old key
    order, and to the linear scan taken from any distance (walk_linear=1e-6), with no light
    buffers too (every shadow ray walks)."""
    if case is None:
        desc, w, h, depth, cam = SceneDesc.synth_config(3), 480, 270, 8, None
    else:
        seed, scale, cam_mode, near, slivers = case
        desc, w, h, depth = stress_scene(seed, scale, near, slivers), 160, 120, 8
        cam = stress_camera(w, h, scale, cam_mode)
    out = []
    for tune in (None, "walk_linear=0", "walk_first=0,walk_linear=0", "walk_linear=0.000001",
                 "lb_res=0,walk_linear=0.000001"):
        s = DeviceScene(desc, device=0, tuning=tune)
        out.append(s.render(w, h, depth, cam=cam)[:2])
        s.close()
    for img, cnt in out[1:]:
        assert same_bits(img, out[0][0]) and cnt == out[0][1]


@pytest.mark.parametrize("key", ["18", "cell", "16"])
def test_shadow_queue_order_changes_nothing(key, monkeypatch):
    """The shadow queue's sort key (default: light | light-buffer cell | distance) only
    orders the queue: frames and counters equal every other ordering bit for bit."""
    desc = SceneDesc.synth_config(3)
    s = DeviceScene(desc, device=0)
    ref, rcnt, _, _ = s.render(320, 180, 8)
    s.close()
    s = DeviceScene(desc, device=0, tuning=f"shadow_key={key}")
    img, cnt, _, _ = s.render(320, 180, 8)
    s.close()
    assert same_bits(img, ref) and cnt == rcnt


def _lights_at_the_edges(seed, scale):
    """A stress scene plus point lights placed around the light buffers' absolute constants
    (DESIGN.md §4.3): at 0.5 - 3 x rho = 0.05 from a sphere's surface (no buffer below rho,
    the nearest records in the all-cell leaves above it), and at 0.8 - 1.3 x the tiers' reach
    Lambda = 45 * 2^t from the scene (the tier boundaries)."""
    d = stress_scene(seed, scale, False, seed % 2 == 0)
    rng = np.random.default_rng(1000 + seed)
    for k in range(3):
        c, r = d.stress_spheres[int(rng.integers(0, 140))]
        u = rng.normal(size=3)
        u /= np.linalg.norm(u)
        gap = float(rng.uniform(0.5, 3.0)) * 0.05
        d.point_light(tuple(c + u * (r * 1.01 + gap)), (0.3, 0.3, 0.3))
    for t in range(2):
        u = rng.normal(size=3)
        u[1] = abs(u[1])
        u /= np.linalg.norm(u)
        reach = 45.0 * 2 ** int(rng.integers(0, 4)) * float(rng.uniform(0.8, 1.3))
        d.point_light(tuple(u * reach), (0.4, 0.4, 0.4))
    return d


@pytest.mark.parametrize("seed,scale", [(40, 1.0), (41, 1.0), (42, 0.1), (43, 0.1), (44, 10.0), (45, 3.0)])
def test_light_buffers_at_their_constants(seed, scale):
    """Lights near the light buffers' absolute constants (rho = 0.05 from a primitive; the
    tiers' reach 45 * 2^t): frames and counters identical with the light buffers (default),
    without them (lb_res=0: every shadow ray walks the hierarchy) and with the linear scan
    (bvh=0: every shape tested for every ray, the reference's Scene::intersect)."""
    desc = _lights_at_the_edges(seed, scale)
    w, h, depth = 160, 120, 6
    cam = stress_camera(w, h, scale, "std")
    out = []
    for tune in (None, "lb_res=0", "bvh=0"):
        s = DeviceScene(desc, device=0, tuning=tune)
        out.append(s.render(w, h, depth, cam=cam)[:2])
        s.close()
    for img, cnt in out[1:]:
        assert same_bits(img, out[0][0]) and cnt == out[0][1]
