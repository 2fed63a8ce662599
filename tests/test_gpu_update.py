"""The drop-in render() keeps one device scene across calls (rt_scene_update).

The reference's render() (src/render.rs:31-38) is called again and again with the same
&Scene -- the bench loop (src/main.rs:137-140) through render_scene_basic (main.rs:244-261)
-- and does no scene preprocessing.  The C++ host mirror's Scene keeps its device handle
across render() calls and brings it up to date with rt_scene_update: nothing when the scene
is unchanged, material edits in place (rt_scene_set_material), a rebuild adopted by the
same handle after any other edit (find_shape_mut + set_transform, mod.rs:66-74; add_light).
Every cached or updated frame must equal, bit for bit, the frame a newly created handle of
the edited scene renders (and that one is checked against the oracle by the parity tests).
"""
import numpy as np
import pytest

from oracle.oracle import OracleScene
from rust_tracer_amd import DeviceScene, Matrix, SceneDesc, abi, mirror_render_calls

pytestmark = pytest.mark.gpu


def same_bits(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("scene", [0, 3])
def test_mirror_render_reuses_the_device_scene(scene):
    """render() x 3 on one Scene: created once, then reused; frames equal rt_render's."""
    w, h, depth = 320, 180, 8
    ms, up, rgb, _ = mirror_render_calls(scene, w, h, depth, 3)
    assert up == [-1, 0, 0], up
    desc = SceneDesc.my_scene() if scene == 0 else SceneDesc.synth_config(scene)
    ref, _, _, _ = DeviceScene(desc, device=0).render(w, h, depth)
    assert same_bits(rgb, ref)
    # a reused handle costs a frame, not a scene build
    assert ms[2] < ms[0], ms


@pytest.mark.parametrize("edit,kind", [(1, 2), (2, 1), (3, 2)])
@pytest.mark.parametrize("scene", [0, 3])
def test_mirror_render_after_edit_equals_fresh_handle(scene, edit, kind):
    """set_transform (rebuild), a material edit (in place), add_light (rebuild, more lights):
    the cached handle's frame after the edit equals a fresh handle's bit for bit."""
    w, h, depth = 320, 180, 8
    _, up0, before, _ = mirror_render_calls(scene, w, h, depth, 2)
    ms, up, rgb, fresh = mirror_render_calls(scene, w, h, depth, 3, edit=edit, fresh=True)
    assert up == [-1, 0, kind], up
    assert same_bits(rgb, fresh)
    assert not same_bits(rgb, before), "the edit changed nothing"


def _edited(desc):
    d = desc.editable()
    sph = next(i for i, s in enumerate(d.shapes) if s.kind == 0)
    t = Matrix.translate(0.0, 0.15, 0.0)
    cur = Matrix([[d.shapes[sph].transform[4 * r + c] for c in range(4)] for r in range(4)])
    d.shapes[sph].transform[:] = (t * cur).flat()
    return d


def test_update_kinds_and_every_render_path():
    """DeviceScene.update: unchanged / materials / rebuilt; after a rebuild rt_render (two band
    shares: the split clones adopt the new scene), a stream-ordered frame and a multi-device
    handle all equal fresh handles of the edited scene, and the oracle."""
    import torch
    w, h, depth = 256, 144, 8
    base = SceneDesc.synth_config(3).editable()
    s = DeviceScene(base, device=0)
    s.render(w, h, depth)
    assert s.update(base) == "unchanged"
    d2 = _edited(base)
    assert s.update(d2) == "rebuilt"
    got, cnt, _, _ = s.render(w, h, depth)
    want, wcnt, _, _ = DeviceScene(d2, device=0).render(w, h, depth)
    assert same_bits(got, want) and cnt == wcnt
    # material edit in place
    d3 = _edited(base)
    d3.materials[0].reflectivity = float(np.float32(d3.materials[0].reflectivity + 0.1))
    assert s.update(d3) == "materials"
    got3, _, _, _ = s.render(w, h, depth)
    want3, _, _, _ = DeviceScene(d3, device=0).render(w, h, depth)
    assert same_bits(got3, want3)
    # stream-ordered frame on the updated handle
    stream = torch.cuda.Stream()
    d_rgb = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda:0")
    cam = abi.camera(w, h)
    s.render_frame_async(cam, depth, d_rgb.data_ptr(), 0, stream.cuda_stream)
    s.sync_status()
    assert same_bits(d_rgb.cpu().numpy(), want3)
    # a multi-device handle (one GPU listed twice: band shares exchanged by device copies)
    m = DeviceScene(base, devices=[0, 0])
    m.render(w, h, depth)
    assert m.update(d3) == "rebuilt"
    gotm, _, _, _ = m.render(w, h, depth)
    assert same_bits(gotm, want3)
    # the oracle on a few rows of the edited scene (rt_render vs the reference restatement)
    ref, _ = OracleScene(d3).render(w, h, depth, rows=(0, h, 24))
    assert np.abs(got3[::24].astype(np.float64) - ref[::24].astype(np.float64)).max() <= 1e-4


def test_update_error_keeps_the_previous_scene():
    """A singular transform (matrix.rs:116-117's panic) is RT_ERR_SINGULAR_MATRIX from
    rt_scene_update; the handle keeps rendering its previous scene."""
    from rust_tracer_amd import RtError
    w, h, depth = 128, 96, 4
    base = SceneDesc.my_scene().editable()
    s = DeviceScene(base, device=0)
    before, _, _, _ = s.render(w, h, depth)
    bad = _edited(base)
    bad.shapes[0].transform[:] = [0.0] * 16
    with pytest.raises(RtError) as e:
        s.update(bad)
    assert e.value.status == 2
    after, _, _, _ = s.render(w, h, depth)
    assert same_bits(after, before)


def test_size_check_refused_inside_stream_capture():
    """The first pass of a new size waits on the host (rt_api.h "HOST WAIT"); inside a stream
    capture it returns RT_ERR_UNSUPPORTED and enqueues nothing, instead of breaking the
    capture with a host synchronisation."""
    import torch
    from rust_tracer_amd import RtError
    s = DeviceScene(SceneDesc.my_scene(), device=0)
    w, h, depth = 64, 48, 4
    d_rgb = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda:0")  # one band share = the frame
    stream = torch.cuda.Stream()
    cam = abi.camera(w, h)
    # warm-up outside the capture at this size: the workspace exists and this size is checked
    s.render_bands_ex_async([cam], depth, 8, 0, 1, d_rgb.data_ptr(), 0, 0, stream.cuda_stream)
    s.sync_status()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    err = None
    with torch.cuda.graph(g, stream=stream, capture_error_mode="relaxed"):
        try:  # a deeper pass than any checked one: refused
            s.render_bands_ex_async([cam], depth + 4, 8, 0, 1, d_rgb.data_ptr(), 0, 0, stream.cuda_stream)
        except RtError as e:
            err = e.status
    assert err == 3, err
    torch.cuda.synchronize()
    # outside the capture the same pass runs (and is checked)
    s.render_bands_ex_async([cam], depth + 4, 8, 0, 1, d_rgb.data_ptr(), 0, 0, stream.cuda_stream)
    s.sync_status()


def test_multi_handle_material_edit_and_revert():
    """A material edit in place on a multi-device handle, then reverted (a GUI slider A -> B ->
    A): the handle records each edit, so the revert is applied too -- every frame equals a fresh
    handle of the same description (the multi branch used to skip the record)."""
    w, h, depth = 192, 108, 6
    base = SceneDesc.synth_config(3).editable()
    m = DeviceScene(base, devices=[0, 0])
    a, _, _, _ = m.render(w, h, depth)
    edited = SceneDesc.synth_config(3).editable()
    k = next(s.material for s in edited.shapes if s.kind == 0)  # the first sphere's material
    mat = edited.materials[k]
    mat.diffuse.color.r = float(np.float32(mat.diffuse.color.r * 0.5))
    mat.reflectivity = float(np.float32(0.7 if mat.reflectivity < 0.6 else 0.2))
    assert m.update(edited) == "materials"
    b, _, _, _ = m.render(w, h, depth)
    want_b, _, _, _ = DeviceScene(edited, device=0).render(w, h, depth)
    assert same_bits(b, want_b) and not same_bits(b, a)
    assert m.update(base) == "materials"
    c, _, _, _ = m.render(w, h, depth)
    assert same_bits(c, a)


def test_forest_refuses_to_shade_after_rebuild():
    """A forest made before a rebuild keeps its trees (sizes, ids) but refuses to shade them
    with the new scene (RT_ERR_INVALID_ARG); a material edit in place keeps it valid."""
    from rust_tracer_amd import RtError
    base = SceneDesc.my_scene().editable()
    s = DeviceScene(base, device=0)
    f = s.forest(64, 48, 4)
    img = f.render()
    sizes = f.tree_sizes()
    d2 = base.editable()
    d2.materials[0].reflectivity = float(np.float32(d2.materials[0].reflectivity + 0.25))
    assert s.update(d2) == "materials"
    f.render()  # in-place edits: the forest shades with them
    d3 = _edited(d2)
    assert s.update(d3) == "rebuilt"
    with pytest.raises(RtError) as e:
        f.render()
    assert e.value.status == 1
    with pytest.raises(RtError):
        f.render_filter([0], img)
    assert np.array_equal(f.tree_sizes(), sizes)
    g = s.forest(64, 48, 4)  # a new forest of the rebuilt scene shades
    assert g.render().shape == img.shape
    g.close()
    f.close()
