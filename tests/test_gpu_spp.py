"""GPU parity of the supersampled render (BASELINE config 5: 64 jittered samples per
pixel, seed 3; rt_render_spp, include/rt_api.h).  The reference has no supersampling
(SURVEY.md §7 step 6), so parity is against the oracle evaluating the same jitter hash
and the same sample-order f32 sum; tolerance 1e-4 per channel as for render.rs."""
import numpy as np
import os
import pytest

from oracle.oracle import OracleScene
from rust_tracer_amd import DeviceScene, RtError, SceneDesc
from tests.test_gpu_parity import compare

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_spp1_is_render():
    s = DeviceScene(SceneDesc.my_scene())
    a, ca, _, _ = s.render(64, 48, 8)
    b, cb, _, _ = s.render(64, 48, 8, spp=1, seed=9)
    s.close()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and ca == cb


def test_spp_golden_fixture():
    g = np.load(os.path.join(GOLDEN, "spp_small.npz"))
    s = DeviceScene(SceneDesc.my_scene())
    img, cnt, _, _ = s.render(32, 32, 4, spp=4, seed=3)
    s.close()
    compare(img, g["rgb_my_scene"])
    assert [cnt["node_rays"], cnt["shadow_rays"], cnt["pixels"]] == list(g["counters_my_scene"])
    s = DeviceScene(SceneDesc.synth_config(5))
    img, cnt, _, _ = s.render(48, 27, 8, spp=4, seed=3)
    s.close()
    compare(img, g["rgb_c5"])
    assert [cnt["node_rays"], cnt["shadow_rays"], cnt["pixels"]] == list(g["counters_c5"])


@pytest.mark.parametrize("spp,seed", [(2, 0), (7, 3), (16, 12345)])
def test_spp_vs_oracle(spp, seed):
    desc = SceneDesc.synth_config(5)
    s = DeviceScene(desc)
    img, cnt, _, _ = s.render(80, 45, 8, spp=spp, seed=seed)
    s.close()
    ref, rcnt = OracleScene(desc).render(80, 45, 8, spp=spp, seed=seed, threads=16)
    compare(img, ref)
    assert cnt == rcnt and cnt["pixels"] == 80 * 45 * spp


def test_config5_4k_sampled_rows():
    """3840x2160 depth 8 (config 5's frame) at 8 samples per pixel: two rows against the
    oracle, the whole frame run-to-run identical."""
    desc = SceneDesc.synth_config(5)
    s = DeviceScene(desc)
    img, cnt, _, _ = s.render(3840, 2160, 8, spp=8, seed=3)
    img2, cnt2, _, _ = s.render(3840, 2160, 8, spp=8, seed=3)
    s.close()
    assert np.array_equal(img.view(np.uint32), img2.view(np.uint32)) and cnt == cnt2
    assert cnt["pixels"] == 3840 * 2160 * 8
    rows = (1001, 2160, 1000)
    ref, _ = OracleScene(desc).render(3840, 2160, 8, rows=rows, threads=2, spp=8, seed=3)
    r = np.arange(*rows)
    compare(img[r], ref[r])


def test_config5_64spp_every_64th_row():
    """Config 5 as benchmarked: 3840x2160, depth 8, 64 jittered samples per pixel, seed 3.
    Every 64th row (34 rows x 3840 pixels x 64 samples) against the oracle, ray counters
    included: rank 0 of a 64-rank band split with 1-row bands is exactly rows 0, 64, 128, ...,
    so its band render gives those rows' own counters -- and equals the whole frame's rows
    bit for bit.  Reference per sample: render.rs:178-185 (get_ray) and :40-103."""
    import torch
    from rust_tracer_amd import abi, band_rows_per_rank
    from tests.test_gpu_fullframe import host_threads
    desc = SceneDesc.synth_config(5)
    w, h, spp, seed, world = 3840, 2160, 64, 3, 64
    s = DeviceScene(desc)
    img, cnt, _, _ = s.render(w, h, 8, spp=spp, seed=seed)
    assert cnt["pixels"] == w * h * spp
    rpr = band_rows_per_rank(h, 1, world)
    dev = torch.device("cuda", 0)
    band = torch.zeros((rpr, w, 3), dtype=torch.float32, device=dev)
    bcnt = torch.zeros(3, dtype=torch.int64, device=dev)
    s.render_bands_async(abi.camera(w, h), 8, 1, 0, world, band.data_ptr(), bcnt.data_ptr(),
                         torch.cuda.current_stream(dev).cuda_stream, spp=spp, seed=seed)
    torch.cuda.synchronize()
    s.sync_status()
    s.close()
    rows = np.arange(0, h, world)
    band = band.cpu().numpy()[:len(rows)]
    assert np.array_equal(band.view(np.uint32), img[rows].view(np.uint32))
    ref, rcnt = OracleScene(desc).render(w, h, 8, rows=(0, h, world), threads=host_threads(), spp=spp, seed=seed)
    compare(band, ref[rows])
    assert rcnt["pixels"] == len(rows) * w * spp
    assert bcnt.cpu().tolist() == [rcnt["node_rays"], rcnt["shadow_rays"], rcnt["pixels"]]


def test_spp_bands_reassemble():
    """The multi-GPU band path with samples: per-rank bands + unpermute == one launch."""
    import torch
    from rust_tracer_amd import abi, band_rows_per_rank, unpermute_bands_async
    desc = SceneDesc.synth_config(5)
    w, h, depth, spp = 120, 70, 8, 5
    s = DeviceScene(desc)
    full, cnt, _, _ = s.render(w, h, depth, spp=spp, seed=3)
    cam = abi.camera(w, h)
    world = 3
    rpr = band_rows_per_rank(h, 8, world)
    bufs = torch.zeros((world, rpr, w, 3), dtype=torch.float32, device="cuda")
    counters = torch.zeros(3, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for r in range(world):
        s.render_bands_async(cam, depth, 8, r, world, bufs[r].data_ptr(), counters.data_ptr(), stream,
                             spp=spp, seed=3)
    frame = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
    unpermute_bands_async(bufs.data_ptr(), w, h, 8, world, frame.data_ptr(), stream)
    torch.cuda.synchronize()
    assert np.array_equal(frame.cpu().numpy().view(np.uint32), full.view(np.uint32))
    assert counters.cpu().tolist() == [cnt["node_rays"], cnt["shadow_rays"], cnt["pixels"]]
    s.close()


def test_spp_zero_rejected():
    s = DeviceScene(SceneDesc.my_scene())
    with pytest.raises(RtError):
        s.render(8, 8, 2, spp=0)
    s.close()


@pytest.mark.parametrize("keys", ["mix", "mixfine", "frame"])
def test_sample_batches_change_nothing(monkeypatch, keys):
    """Samples batched B per pipeline pass (each a frame of the pass with its own jitter,
    summed in sample order by spp_accumulate_kernel) equal one pass per sample
    (spp_batch=1) bit for bit, RGB8 included -- 19 samples: batches of 8, 8 and 3, so the
    running sum crosses batches and the last batch is partial; every queue-key variant."""
    desc = SceneDesc.synth_config(5)
    w, h, spp = 160, 90, 19
    s = DeviceScene(desc, device=0, tuning="spp_batch=1")
    ref, rcnt, _, ref8 = s.render(w, h, 8, spp=spp, seed=3, want_u8=True)
    s.close()
    s = DeviceScene(desc, device=0, tuning=f"spp_batch=8,spp_keys={keys}")
    img, cnt, _, img8 = s.render(w, h, 8, spp=spp, seed=3, want_u8=True)
    s.close()
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(img8, ref8) and cnt == rcnt


def test_sample_batches_in_bands(monkeypatch):
    """A band share (rank 1 of 3) of a supersampled frame: batched samples equal one pass per
    sample (the multi-GPU path of config 5)."""
    import torch
    from rust_tracer_amd import abi, band_rows_per_rank
    desc = SceneDesc.synth_config(5)
    w, h, spp, world = 200, 117, 10, 3
    dev = torch.device("cuda", 0)
    rpr = band_rows_per_rank(h, 8, world)
    outs = []
    for b in ("1", "4"):
        s = DeviceScene(desc, device=0, tuning=f"spp_batch={b}")
        out = torch.full((rpr, w, 3), -1.0, device=dev)
        cnt = torch.zeros(3, dtype=torch.int64, device=dev)
        s.render_bands_async(abi.camera(w, h), 8, 8, 1, world, out.data_ptr(), cnt.data_ptr(),
                             torch.cuda.current_stream(dev).cuda_stream, spp=spp, seed=3)
        torch.cuda.synchronize()
        s.sync_status()
        outs.append((out.cpu().numpy(), cnt.cpu().numpy()))
        s.close()
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1], outs[1][1])
