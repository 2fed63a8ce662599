"""GPU tests of the drop-in seam beyond one device and one float frame:

- multi-device scenes (rt_scene_create_multi): the frame tiled over ranks, gathered and
  un-permuted, equals the one-device rt_render bit for bit -- with one GPU listed 2 / 3 times
  (band shares exchanged by device copies: the multi-rank band logic on a one-GPU box), and
  with tuning force_rccl=1 and one device: a one-rank RCCL communicator (ncclCommInitAll), the
  grouped ncclGather and the un-permute kernel really execute on the one-GPU box;
- bench.py under torchrun --nproc-per-node 1 --backend nccl --force-gather 1: the
  process-group path's RCCL gather (torch.distributed over RCCL) with frame_check;
- queue overflow is never a silent RT_OK: the stream-ordered entry points latch it and
  rt_scene_sync_status raises RT_ERR_CAPACITY; rt_render grows its pool and renders the
  full frame (render.rs:40-103 traces every ray);
- Color::as_u8 fused into the level-0 combine (color.rs:43-46): RGB8 equals as_u8 of the
  float frame on every path (rt_render, band renders, RGB8-only band renders, multi-device);
- BASELINE config 4 (3840x2160, depth 8, 1 spp) against the oracle on sampled rows.
"""
import os

import numpy as np
import pytest
import torch

from oracle.oracle import OracleScene, as_u8
from rust_tracer_amd import DeviceScene, RtError, SceneDesc, abi, band_rows_per_rank
from rust_tracer_amd.dist import local_rows

pytestmark = pytest.mark.gpu

TOL = 1e-4


def same_bits(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def compare(gpu, ref, tol=TOL):
    diff = np.abs(gpu.astype(np.float64) - ref.astype(np.float64))
    diff[np.isnan(gpu) & np.isnan(ref)] = 0.0
    assert not np.isnan(diff).any(), "NaN in one image only"
    assert float(diff.max()) <= tol


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_multi_device_scene_equals_single(devices):
    """rt_scene_create_multi: same frame, counters and RGB8 as the one-device render."""
    desc = SceneDesc.synth_config(3)
    w, h, depth = 320, 180, 8
    single = DeviceScene(desc, device=0)
    ref, rcnt, _, ref8 = single.render(w, h, depth, want_u8=True)
    single.close()
    multi = DeviceScene(desc, devices=devices)
    assert multi.device_count == len(devices)
    # without force_rccl, one device is a plain scene and a repeated device exchanges
    # bands by device copies: no RCCL
    assert not multi.uses_rccl
    img, cnt, ms, img8 = multi.render(w, h, depth, want_u8=True)
    img2, cnt2, _, _ = multi.render(w, h, depth)  # buffers reused
    multi.close()
    assert same_bits(img, ref) and same_bits(img2, ref)
    assert np.array_equal(img8, ref8)
    assert cnt == rcnt and cnt2 == rcnt
    assert ms > 0


def test_multi_device_eight_ranks_config4():
    """The N = 8 band layout behind the drop-in seam: rt_scene_create_multi with devices =
    [0] * 8 (eight band shares of one GPU, exchanged by device copies) renders the whole
    config 4 frame (3840x2160, depth 8) bit-identical to the one-device rt_render, counters
    equal -- the driver's 8-GPU run deals the same bands to eight devices (render.rs:32-37
    tiled)."""
    desc = SceneDesc.synth_config(4)
    single = DeviceScene(desc, device=0)
    ref, rcnt, _, _ = single.render(3840, 2160, 8)
    single.close()
    multi = DeviceScene(desc, devices=[0] * 8)
    assert multi.device_count == 8
    img, cnt, _, _ = multi.render(3840, 2160, 8)
    multi.close()
    assert same_bits(img, ref)
    assert cnt == rcnt


@pytest.mark.parametrize("w,h", [(320, 180), (3840, 2160)])
def test_forced_rccl_one_rank(monkeypatch, w, h):
    """Tuning force_rccl=1 (RT_TUNE) with devices=[0]: rt_scene_create_multi builds a one-rank RCCL
    communicator, and rt_render runs the band render, the grouped ncclGather (rt_multi.cpp)
    and the un-permute kernel.  Config 3 at 320x180 and the whole config 4 frame (3840x2160,
    depth 8) equal the one-device rt_render bit for bit (render.rs:32-37 tiled)."""
    desc = SceneDesc.synth_config(3)
    single = DeviceScene(desc, device=0)
    ref, rcnt, _, ref8 = single.render(w, h, 8, want_u8=True)
    single.close()
    monkeypatch.setenv("RT_TUNE", "force_rccl=1")
    multi = DeviceScene(desc, devices=[0])
    assert multi.uses_rccl and multi.device_count == 1
    img, cnt, ms, img8 = multi.render(w, h, 8, want_u8=True)
    img2, cnt2, _, _ = multi.render(w, h, 8)  # communicator and buffers reused
    multi.close()
    assert same_bits(img, ref) and same_bits(img2, ref)
    assert np.array_equal(img8, ref8)
    assert cnt == rcnt and cnt2 == rcnt
    assert ms > 0


def test_forced_rccl_overflow_rerenders(monkeypatch):
    """A one-rank RCCL scene whose node pool is far too small: the rank re-renders with a
    grown pool, the gather runs again, and the frame is complete."""
    desc = SceneDesc.synth_config(3)
    single = DeviceScene(desc, device=0)
    ref, rcnt, _, _ = single.render(256, 144, 8)
    single.close()
    monkeypatch.setenv("RT_TUNE", f"force_rccl=1,node_cap={256 * 144 + 4096}")
    multi = DeviceScene(desc, devices=[0])
    assert multi.uses_rccl
    img, cnt, _, _ = multi.render(256, 144, 8)
    multi.close()
    assert same_bits(img, ref) and cnt == rcnt


def test_torchrun_one_rank_nccl_gather():
    """bench.py under torchrun with one rank, backend nccl (RCCL) and --force-gather 1: every
    pass is assembled through torch.distributed.gather over a one-rank RCCL communicator and
    the un-permute kernel (dist.py FrameTiler.assemble), and frame_check holds."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29613", "bench.py", "--backend", "nccl",
           "--force-gather", "1", "--check", "1", "--steps", "4", "--warmup", "1", "--inflight", "2",
           "--cpu-baseline", "0", "--count-frame", "0", "--seam-stats", "0"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 1
    assert out["frame_check"] is True and out["frame_check_frames"] >= 3


def test_pipeline_overflow_is_raised(monkeypatch):
    """FramePipeline with a node pool far too small: frames() raises RT_ERR_CAPACITY instead
    of returning incomplete frames; the slots' next passes get grown pools and are complete."""
    from rust_tracer_amd.dist import FramePipeline
    desc = SceneDesc.synth_config(3)
    w, h, depth = 192, 108, 8
    ref_scene = DeviceScene(desc, device=0)
    ref, _, _, _ = ref_scene.render(w, h, depth)
    ref_scene.close()
    s = DeviceScene(desc, device=0, tuning=f"node_cap={w * h + 1024}")  # the clones copy it
    pipe = FramePipeline(s, desc, w, h, depth, inflight=2, batch=1)
    pipe.run(2)
    torch.cuda.synchronize()
    # every slot's pass overflowed and each reports it (rt_scene_sync_status per slot)
    for t in pipe.tilers:
        with pytest.raises(RtError) as e:
            t.scene.sync_status()
        assert e.value.status == abi.RT_ERR_CAPACITY
    pipe.run(2)
    with pytest.raises(RtError) as e:
        pipe.frames()
    assert e.value.status == abi.RT_ERR_CAPACITY
    for attempt in range(6):  # each reported overflow doubles that slot's pool
        pipe.run(2)
        try:
            frames = pipe.frames()
            break
        except RtError as e:
            assert e.status == abi.RT_ERR_CAPACITY
    assert len(frames) == 2 and all(same_bits(f.cpu().numpy(), ref) for f in frames)
    pipe.close()
    assert s.grid_share == 100  # the caller's scene gets its grid share back
    s.close()


def test_multi_device_ragged_and_spp():
    """Frames whose rows do not fill the last bands, and jittered supersampling, tiled."""
    desc = SceneDesc.my_scene()
    single = DeviceScene(desc, device=0)
    multi = DeviceScene(desc, devices=[0, 0, 0])
    for (w, h, spp) in [(67, 45, 1), (8, 3, 1), (96, 61, 4)]:
        ref, rcnt, _, _ = single.render(w, h, 6, spp=spp, seed=7)
        img, cnt, _, _ = multi.render(w, h, 6, spp=spp, seed=7)
        assert same_bits(img, ref), (w, h, spp)
        assert cnt == rcnt
    single.close()
    multi.close()


def test_scene_clone_renders_identically():
    desc = SceneDesc.synth_config(2)
    a = DeviceScene(desc, device=0)
    b = a.clone(0)
    ra, ca, _, _ = a.render(200, 120, 4)
    rb, cb, _, _ = b.render(200, 120, 4)
    assert same_bits(ra, rb) and ca == cb
    b.close()
    ra2, _, _, _ = a.render(200, 120, 4)  # the source outlives its clone
    assert same_bits(ra, ra2)
    a.close()


def _band_render(scene, w, h, depth, rank, world, rgb=True, rgb8=False, band_rows=8):
    dev = torch.device("cuda", 0)
    rpr = band_rows_per_rank(h, band_rows, world)
    out = torch.full((rpr, w, 3), -1.0, dtype=torch.float32, device=dev) if rgb else None
    out8 = torch.zeros((rpr, w, 3), dtype=torch.uint8, device=dev) if rgb8 else None
    cnt = torch.zeros(3, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    scene.render_bands_ex_async([abi.camera(w, h)], depth, band_rows, rank, world,
                                out.data_ptr() if rgb else 0, out8.data_ptr() if rgb8 else 0, cnt.data_ptr(),
                                stream)
    torch.cuda.synchronize()
    return (out.cpu().numpy() if rgb else None), (out8.cpu().numpy() if rgb8 else None), cnt.cpu().numpy()


def test_overflow_is_reported_not_truncated(monkeypatch):
    """A node pool far too small for the ray trees: the stream-ordered render still returns
    RT_OK (it cannot know yet), rt_scene_sync_status then raises RT_ERR_CAPACITY; the next
    pass gets a grown pool.  rt_render retries internally and returns the full frame."""
    desc = SceneDesc.synth_config(3)
    w, h, depth = 256, 144, 8
    full = DeviceScene(desc, device=0)
    ref, rcnt, _, _ = full.render(w, h, depth)
    full.close()
    s = DeviceScene(desc, device=0, tuning=f"node_cap={w * h + 4096}")  # level 0 plus a sliver
    _band_render(s, w, h, depth, 0, 1)
    with pytest.raises(RtError) as e:
        s.sync_status()
    assert e.value.status == abi.RT_ERR_CAPACITY
    s.sync_status()  # cleared once reported
    # rt_render grows the pool until every ray fits
    img, cnt, _, _ = s.render(w, h, depth)
    assert same_bits(img, ref) and cnt == rcnt
    s.close()
    s = DeviceScene(desc, device=0)
    _band_render(s, w, h, depth, 0, 1)
    s.sync_status()  # default pool: no overflow
    s.close()


@pytest.mark.parametrize("world", [1, 3])
def test_fused_rgb8_bands(world):
    """RGB8 written by the level-0 combine equals as_u8 of the float bands; RGB8-only bands
    (no float frame written) are the same bytes."""
    desc = SceneDesc.my_scene()
    w, h, depth = 130, 77, 8
    s = DeviceScene(desc, device=0)
    for rank in range(world):
        f, b8, c = _band_render(s, w, h, depth, rank, world, rgb=True, rgb8=True)
        assert np.array_equal(b8, as_u8(f))
        _, only8, c2 = _band_render(s, w, h, depth, rank, world, rgb=False, rgb8=True)
        assert np.array_equal(only8, b8)
        assert np.array_equal(c, c2)
    s.sync_status()
    s.close()


def test_u8_unpermute_matches_float_unpermute():
    from rust_tracer_amd import unpermute_bands_async, unpermute_bands_u8_async
    dev = torch.device("cuda", 0)
    w, h, br, world = 37, 53, 8, 3
    rpr = band_rows_per_rank(h, br, world)
    g = torch.rand((world, rpr, w, 3), device=dev)
    g8 = (g * 255).to(torch.uint8)
    f = torch.zeros((h, w, 3), device=dev)
    f8 = torch.zeros((h, w, 3), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    unpermute_bands_async(g.data_ptr(), w, h, br, world, f.data_ptr(), st)
    unpermute_bands_u8_async(g8.data_ptr(), w, h, br, world, f8.data_ptr(), st)
    torch.cuda.synchronize()
    assert torch.equal((f * 255).to(torch.uint8), f8)
    for r in range(world):
        for lr, v in enumerate(local_rows(h, br, r, world)):
            if v >= 0:
                assert torch.equal(f8[v], g8[r, lr])


def test_config4_sampled_rows():
    """BASELINE config 4: 3840x2160, depth 8, 1 spp, the config-3 scene; rows sampled across
    the frame (every 270th) against the oracle, and the whole frame run-to-run identical."""
    desc = SceneDesc.synth_config(4)
    s = DeviceScene(desc, device=0)
    img, cnt, _, img8 = s.render(3840, 2160, 8, want_u8=True)
    img2, cnt2, _, _ = s.render(3840, 2160, 8)
    s.close()
    assert cnt["pixels"] == 3840 * 2160 and cnt == cnt2
    assert same_bits(img, img2)
    assert np.array_equal(img8, as_u8(img))
    rows = np.arange(13, 2160, 270)
    ref, _ = OracleScene(desc).render(3840, 2160, 8, rows=(13, 2160, 270), threads=16)
    compare(img[rows], ref[rows])


def test_config4_tiled_two_ways():
    """Config 4 tiled over ranks through the C ABI (one GPU listed twice) equals the whole
    frame rendered on one device."""
    desc = SceneDesc.synth_config(4)
    s = DeviceScene(desc, device=0)
    ref, rcnt, _, _ = s.render(3840, 2160, 8)
    s.close()
    m = DeviceScene(desc, devices=[0, 0])
    img, cnt, _, _ = m.render(3840, 2160, 8)
    m.close()
    assert same_bits(img, ref) and cnt == rcnt


def test_torchrun_two_ranks_render_and_gather():
    """bench.py under torchrun with two ranks (gloo exchange on one GPU): every rank renders
    its bands of config 3, rank 0 gathers and un-permutes, and the assembled frames equal a
    single-launch render bit for bit (frame_check)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29611", "bench.py", "--backend", "gloo", "--check", "1",
           "--steps", "2", "--warmup", "1", "--inflight", "2", "--cpu-baseline", "0", "--count-frame", "0",
           "--seam-stats", "0"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2
    assert out["frame_check"] is True


def _axis_scene():
    """A sphere on the camera axis with a point light straight behind it: the centre pixel's
    eye direction and its (shadowed) light direction are exact opposites, so the reference's
    half vector norm(eye + l) is 0 / 0 and the pixel is NaN (phong, material.rs:197-213)."""
    from rust_tracer_amd import Matrix
    d = SceneDesc()
    red = d.phong((0.1, 0.0, 0.0), (1, 0, 0), (1, 1, 1), 60.0, 0.0, 0.0)
    glass = d.phong((0, 0, 0), (1, 1, 1), (1, 1, 1), 60.0, 0.7, 1.333)
    d.sphere(red, Matrix.identity())
    d.sphere(glass, Matrix.translate(2.0, 1.0, 0.0) * Matrix.scale(0.5, 0.5, 0.5))
    d.point_light((0.0, 0.0, 10.0), (1, 1, 1))
    d.point_light((3.0, 4.0, -6.0), (0.5, 0.5, 0.5))
    d.set_ambient((0.1, 0.1, 0.1))
    return d


@pytest.mark.parametrize("name", ["config3", "my_scene", "axis"])
def test_shadowed_light_skip_is_exact(name, monkeypatch):
    """The combine pass skips shadowed point lights (their term is exactly +-0, light_sum):
    frames equal the full evaluation bit for bit (tuning dark_skip=0), NaNs included."""
    desc = {"config3": lambda: SceneDesc.synth_config(3), "my_scene": SceneDesc.my_scene, "axis": _axis_scene}[name]()
    w, h = (256, 144) if name == "config3" else (64, 64)
    s = DeviceScene(desc, device=0)
    img, cnt, _, _ = s.render(w, h, 8)
    s.close()
    s = DeviceScene(desc, device=0, tuning="dark_skip=0")
    ref, rcnt, _, _ = s.render(w, h, 8)
    s.close()
    assert same_bits(img, ref) and cnt == rcnt
    if name == "axis":
        assert np.isnan(img[32, 32]).all()  # the reference's 0 / 0 half vector
        oimg, ocnt = OracleScene(desc).render(w, h, 8)
        compare(img, oimg)
        assert cnt == ocnt


def _scaled_plane_scene():
    """A floor plane whose transform scales its normal to length 2 (plane.rs:75 shades with
    transform * normal, not normalised) and a specular power of 500: (m.h)^power overflows to
    inf, so a shadowed light's term is inf * BLACK = NaN in the reference (material.rs:211) --
    the combine's shadowed-light skip must not apply there."""
    from rust_tracer_amd import Matrix
    d = SceneDesc()
    floor = d.phong((0.1, 0.1, 0.1), (0.5, 0.5, 0.5), (1, 1, 1), 500.0, 0.0, 0.0)
    ball = d.phong((0.1, 0.0, 0.0), (1, 0, 0), (1, 1, 1), 60.0, 0.0, 0.0)
    d.plane(floor, (0.0, -1.0, 0.0), (0.0, 1.0, 0.0), Matrix.scale(2.0, 2.0, 2.0))
    d.sphere(ball, Matrix.translate(0.0, -1.0, 0.0) * Matrix.scale(0.6, 0.6, 0.6))
    d.point_light((0.0, 10.0, 0.0), (1, 1, 1))
    d.point_light((3.0, 6.0, -4.0), (0.5, 0.5, 0.5))
    d.set_ambient((0.1, 0.1, 0.1))
    return d


def test_scaled_plane_normal_high_power():
    """Shadowed light on a plane with |transform * n| = 2 and power 500: NaN / inf exactly as
    the oracle and as the full evaluation (tuning dark_skip=0)."""
    desc = _scaled_plane_scene()
    w, h = 96, 96
    s = DeviceScene(desc, device=0)
    img, cnt, _, _ = s.render(w, h, 4)
    s.close()
    ref, rcnt = OracleScene(desc).render(w, h, 4)
    assert cnt == rcnt
    assert np.isnan(ref).any()  # the scene really reaches the inf * BLACK case
    nan_g, nan_r = np.isnan(img), np.isnan(ref)
    assert np.array_equal(nan_g, nan_r)
    eq = img.view(np.uint32) == ref.view(np.uint32)
    differ = ~(eq | (nan_g & nan_r))  # masked before subtracting (equal infinities: inf - inf)
    d = np.zeros(img.shape)
    d[differ] = np.abs(img[differ].astype(np.float64) - ref[differ].astype(np.float64))
    assert float(d.max()) <= TOL


@pytest.mark.parametrize("depth", [65, 200])
def test_depth_beyond_64(depth):
    """The reference recursion is unbounded (render.rs:40-103); the device accepts depth up to
    RT_MAX_DEPTH (1024) and rt_render stops enqueuing levels once one is empty.  my_scene's
    glass and mirror spheres keep rays alive for many levels."""
    desc = SceneDesc.my_scene()
    s = DeviceScene(desc, device=0)
    img, cnt, _, _ = s.render(48, 36, depth)
    s.close()
    ref, rcnt = OracleScene().render(48, 36, depth)
    compare(img, ref)
    assert cnt == rcnt


def test_depth_limit_is_reported():
    s = DeviceScene(SceneDesc.my_scene(), device=0)
    with pytest.raises(RtError) as e:
        s.render(8, 8, abi.RT_MAX_DEPTH + 1)
    s.close()
    assert e.value.status == 3  # RT_ERR_UNSUPPORTED


@pytest.mark.parametrize("rgb8", [False, True])
def test_frame_pipeline_distinct_cameras(rgb8):
    """FramePipeline with a camera per frame (an animation) in batches of 2 on 2 slots: every
    frame equals rt_render of its own camera (RGB8: its Color::as_u8 bytes)."""
    from rust_tracer_amd.dist import FramePipeline
    desc = SceneDesc.synth_config(3)
    w, h, depth, n = 192, 108, 8, 4
    s = DeviceScene(desc, device=0)

    def cam(i):
        c = abi.camera(w, h)
        c.origin[0] = 0.05 * i
        return c
    refs = [s.render(w, h, depth, cam=cam(i), want_u8=True) for i in range(n)]
    pipe = FramePipeline(s, desc, w, h, depth, inflight=2, batch=2, rgb8=rgb8)
    seen = {}
    for p in range(2):  # two passes of 2 frames: frames 0,1 on slot 0 and 2,3 on slot 1
        pipe.run(2, cameras=cam)
        torch.cuda.synchronize()
        t = pipe.tilers[p]
        for b in range(t.last):
            seen[2 * p + b] = t.frames[b].cpu().numpy()
    for i in range(n):
        img, _, _, img8 = refs[i]
        if rgb8:
            assert np.array_equal(seen[i], img8)
        else:
            assert same_bits(seen[i], img)
    assert not same_bits(refs[0][0], refs[1][0])  # the views really differ
    pipe.close()
    s.close()


def test_torchrun_two_ranks_rgb8_gather():
    """The N > 1 path with --output rgb8: RGB8-only bands gathered (3 B per pixel) and
    un-permuted, equal to as_u8 of a single-launch render."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29612", "bench.py", "--backend", "gloo", "--check", "1",
           "--steps", "2", "--warmup", "1", "--inflight", "2", "--cpu-baseline", "0", "--count-frame", "0",
           "--seam-stats", "0", "--output", "rgb8"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["frame_check"] is True and out["config"]["output"] == "rgb8"


@pytest.mark.parametrize("split,rows", [(2, None), (3, None), (2, "8"), (4, "16")])
def test_seam_split_changes_nothing(monkeypatch, split, rows):
    """rt_render on a one-device scene renders the frame as `split` band shares side by side
    (seam_split, contiguous shares by default, seam_band_rows otherwise): frames, RGB8
    and counters equal the single pass (seam_split=1) bit for bit, including a frame too
    small to split and a ragged height; the share handles follow a material edit."""
    desc = SceneDesc.synth_config(3)
    sizes = [(320, 181), (96, 20)]
    s = DeviceScene(desc, device=0, tuning="seam_split=1")
    refs = [s.render(w, h, 8, want_u8=True) for w, h in sizes]
    s.close()
    s = DeviceScene(desc, device=0, tuning=f"seam_split={split}" + (f",seam_band_rows={rows}" if rows else ""))
    for (w, h), (ref, rcnt, _, ref8) in zip(sizes, refs):
        img, cnt, ms, img8 = s.render(w, h, 8, want_u8=True)
        assert same_bits(img, ref) and np.array_equal(img8, ref8) and cnt == rcnt, (w, h)
    # a material edit reaches every share's handle
    from rust_tracer_amd import phong_material
    m = phong_material((0, 0, 0), (0.9, 0.2, 0.1), (1, 1, 1), 30.0, 0.5, 0.0)
    s.set_material(0, m)
    img, cnt, _, _ = s.render(320, 181, 8)
    s.close()
    one = DeviceScene(desc, device=0, tuning="seam_split=1")
    one.set_material(0, m)
    ref, rcnt, _, _ = one.render(320, 181, 8)
    one.close()
    assert same_bits(img, ref) and cnt == rcnt


def test_adaptive_seam_split_changes_nothing(monkeypatch):
    """rt_render's two band shares meet at a row that follows their finish times (moved 8 rows
    per render within [half, 3/4] of the frame, seam_adapt) and run their grids at a
    reduced share of the chip (seam_grid_pct): every one of a run of renders -- whatever
    row the shares meet at -- equals the single pass bit for bit, RGB8 and counters too."""
    desc = SceneDesc.synth_config(3)
    w, h = 640, 361
    s = DeviceScene(desc, device=0, tuning="seam_split=1")
    ref, rcnt, _, ref8 = s.render(w, h, 8, want_u8=True)
    s.close()
    s = DeviceScene(desc, device=0, tuning="seam_split=2,seam_grid_pct=60")
    for _ in range(12):
        img, cnt, _, img8 = s.render(w, h, 8, want_u8=True)
        assert same_bits(img, ref) and np.array_equal(img8, ref8) and cnt == rcnt
    s.close()


def test_pipeline_glass_heavy_scene_completes():
    """A scene whose ray trees far outgrow the default pool (every sphere a reflective glass
    ball: two children per hit, ~20+ nodes per pixel at depth 8 where node_factor sizes 6):
    the first pass of each frame-in-flight slot is checked (rt_render_bands_ex_async grows the
    pool and renders it again), so FramePipeline returns complete frames, equal to rt_render
    bit for bit, with no overflow reported."""
    from rust_tracer_amd.abi import RT_SHAPE_SPHERE
    from rust_tracer_amd.dist import FramePipeline
    desc = SceneDesc.synth_config(3).editable()
    glass = desc.phong((0.05, 0.05, 0.05), (0.2, 0.3, 0.4), (1.0, 1.0, 1.0), 120.0, 0.8, 1.5)
    for sh in desc.shapes:
        if sh.kind == RT_SHAPE_SPHERE:
            sh.material = glass
    w, h, depth = 240, 136, 8
    ref_scene = DeviceScene(desc, device=0)
    ref, rcnt, _, _ = ref_scene.render(w, h, depth)
    ref_scene.close()
    assert rcnt["node_rays"] > 8 * w * h  # the trees really outgrow the default 6 slots per pixel
    s = DeviceScene(desc, device=0)
    pipe = FramePipeline(s, desc, w, h, depth, inflight=2, batch=2)
    for _ in range(2):
        pipe.run(4)
        frames = pipe.frames()  # raises RtError(RT_ERR_CAPACITY) on an incomplete frame
        assert len(frames) == 4 and all(same_bits(f.cpu().numpy(), ref) for f in frames)
    pipe.close()
    s.close()
