"""GPU parity of the ray-forest path (src/render_tree.rs) against the CPU oracle.

generate_ray_forest / render_forest / render_forest_filter / RayTree::size /
RayForest::trees_with on the device (rt_forest_*) against oracle/rt_oracle.cpp's
restatement of render_tree.rs.  The forest's shading differs from render.rs
(render_tree.rs:214-255: eye_dir as the reflected term's light direction, no diffuse
factor on refraction), so it has its own golden frame (tests/golden/forest_64.npz).
Tolerance as everywhere: |gpu - oracle| <= 1e-4 per channel; tree sizes, ray counts and
tree-membership counts exact.
"""
import os

import numpy as np
import pytest

from oracle.oracle import OracleScene
from rust_tracer_amd import DeviceScene, Matrix, SceneDesc, phong_material, texture_phong_material

from .test_gpu_parity import _custom_scene, compare

pytestmark = pytest.mark.gpu


def both(desc, w, h, depth):
    s = DeviceScene(desc)
    o = OracleScene(desc)
    return s, o, s.forest(w, h, depth), o.forest(w, h, depth)


def test_forest_golden_fixture():
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "forest_64.npz"))
    s = DeviceScene(SceneDesc.my_scene())
    f = s.forest(64, 64, 8)
    compare(f.render(), g["rgb_d8"])
    assert np.array_equal(f.tree_sizes(), g["tree_sizes_d8"])


@pytest.mark.parametrize("depth", [1, 3, 8])
def test_forest_my_scene(depth):
    desc = SceneDesc.my_scene()
    s, o, f, fo = both(desc, 128, 96, depth)
    compare(f.render(), fo.render())
    assert np.array_equal(f.tree_sizes(), fo.tree_sizes())
    # the forest's trees are render.rs's trees: same ray counts
    _, rcnt = OracleScene(desc).render(128, 96, depth)
    assert f.counters() == rcnt


def test_forest_custom_scene_and_cube_ids():
    """Textures, rotated / scaled spheres, cubes (inner-triangle ids 0..11 collide with
    shape ids, cube.rs:93-99), loose triangles, TIR, ties."""
    s, o, f, fo = both(_custom_scene(), 160, 120, 8)
    compare(f.render(), fo.render())
    assert np.array_equal(f.tree_sizes(), fo.tree_sizes())
    for k in range(14):
        assert f.trees_with(k) == fo.trees_with(k), k


def test_forest_config3():
    s, o, f, fo = both(SceneDesc.synth_config(3), 160, 90, 8)
    compare(f.render(), fo.render())
    assert np.array_equal(f.tree_sizes(), fo.tree_sizes())


def test_forest_stats_match_reference_definition():
    s, o, f, fo = both(SceneDesc.my_scene(), 96, 64, 8)
    st = f.stats()
    sizes = np.sort(fo.tree_sizes().ravel())
    n = len(sizes)
    assert st["num_trees"] == n and st["num_intersections"] == int(sizes.sum())
    assert st["smallest_tree"] == sizes[0] and st["largest_tree"] == sizes[-1]
    assert st["median"] == sizes[n // 2]
    assert st["p90"] == sizes[int(np.float32(0.9) * np.float32(n))]


def test_forest_filter_after_material_edit():
    """The GUI flow (gui.rs:163-236): build once, edit materials, re-shade only the trees
    holding the edited shapes; the rest of the frame keeps its old values."""
    desc = _custom_scene()
    s, o, f, fo = both(desc, 160, 120, 8)
    img, ref = f.render(), fo.render()
    compare(img, ref)
    # material 3 ("red", shape 2) and material 4 (textured sphere 0)
    edits = {3: phong_material((0.05, 0.0, 0.0), (0.2, 0.9, 0.3), (0.5, 0.5, 0.5), 30.0, 0.0, 0.0),
             4: texture_phong_material((0.2, 0.2, 0.0), "checkerboard", (0.3, 0.3, 0.3), 90.0, 0.3, 0.0)}
    for k, m in edits.items():
        s.set_material(k, m)
        o.set_material(k, m)
    ids = [0, 2]
    got = f.render_filter(ids, img)
    want = fo.render_filter(ids, ref)
    compare(got, want)
    changed = (got != img).any(axis=2)
    assert changed.any()
    # pixels whose trees do not hold 0 or 2 keep their old values exactly
    mask = np.zeros_like(changed)
    for i in ids:
        mask |= _trees_holding(fo, i)
    assert not changed[~mask].any()
    # a full re-shade agrees with the oracle's full re-shade under the new materials
    compare(f.render(), fo.render())


def _trees_holding(fo, shape_id):
    """pixels whose oracle tree holds `shape_id` (those a filtered re-shade overwrites)"""
    sentinel = np.full((fo.h_res, fo.w, 3), 1e30, np.float32)
    return (fo.render_filter([shape_id], sentinel) != 1e30).any(axis=2)


def test_forest_material_edit_affects_renders_too():
    """rt_scene_set_material is the scene's material: later rt_render calls see it."""
    desc = SceneDesc.my_scene()
    s = DeviceScene(desc)
    o = OracleScene(desc)
    m = phong_material((0.0, 0.0, 0.0), (0.0, 1.0, 0.0), (0.1, 0.1, 0.1), 600.0, 0.4, 0.0)
    s.set_material(1, m)
    o.set_material(1, m)
    img, cnt, _, _ = s.render(96, 64, 8)
    ref, rcnt = o.render(96, 64, 8)
    compare(img, ref)
    assert cnt == rcnt


def test_forest_bvh_off_identical():
    desc = SceneDesc.synth_config(3)
    a = DeviceScene(desc).forest(200, 112, 8).render()
    s = DeviceScene(desc, tuning="bvh=0")
    b = s.forest(200, 112, 8).render()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_set_material_rejects_kind_change():
    from rust_tracer_amd import RtError
    s = DeviceScene(SceneDesc.my_scene())
    with pytest.raises(RtError):  # material 3 of my_scene is a TexturePhong
        s.set_material(3, phong_material((0, 0, 0), (1, 1, 1), (1, 1, 1), 10.0, 0.0, 0.0))


def _threads():
    from .test_gpu_fullframe import host_threads
    return host_threads()


def test_forest_config3_benchmark_frame():
    """The benchmark frame (config 3: 1920x1080, depth 8, 1k primitives) as a ray forest:
    generate_ray_forest + render_forest (render_tree.rs:121-164) against the oracle's forest on
    EVERY pixel (bits equal, or NaN in both), tree sizes and RayForest::trees_with exact; then a
    material edit and render_forest_filter (render_tree.rs:129-145, the GUI's re-shade) on every
    pixel too.  The oracle forest is built over the host threads (~10-20 s on the box)."""
    from .test_gpu_fullframe import report
    desc = SceneDesc.synth_config(3)
    w, h, depth = 1920, 1080, 8
    s = DeviceScene(desc, device=0)
    o = OracleScene(desc)
    f = s.forest(w, h, depth)
    fo = o.forest(w, h, depth, threads=_threads())
    img, ref = f.render(), fo.render()
    worst, bad, nan_eq, msg = report(img, ref)
    assert bad == 0 and nan_eq, msg
    assert np.array_equal(f.tree_sizes(), fo.tree_sizes())
    # the forest's trees are render.rs's trees: the same ray counts as rt_render's frame
    _, rcnt, _, _ = s.render(w, h, depth)
    assert f.counters() == rcnt
    for k in (0, 5, 11, 20, 350, 610, 700, 725, 726):  # spheres (0..11 collide with cube ids), a cube's, triangles, planes
        assert f.trees_with(k) == fo.trees_with(k), k
    # a GUI edit of sphere 20's material, re-shaded through the filter
    k = int(desc.editable().shapes[20].material)
    m = phong_material((0.02, 0.0, 0.05), (0.3, 0.8, 0.2), (0.6, 0.6, 0.6), 90.0, 0.4, 0.0)
    s.set_material(k, m)
    o.set_material(k, m)
    got = f.render_filter([20], img)
    want = fo.render_filter([20], ref)
    worst, bad, nan_eq, msg = report(got, want)
    assert bad == 0 and nan_eq, msg
    assert (got != img).any()
    f.close()
