"""GPU tests of rt_render_bands_direct_async (band shares of one device writing their rows of
whole frames in place) and of FramePipeline's sub-band slot groups (bench.py at K = 20).

- S shares (S scene handles, S streams) over n frames with their own cameras fill the frames
  exactly: every frame equals rt_render of its camera bit for bit (f32 and RGB8), counters
  sum to the whole frames', at a ragged size whose last band is padded past the frame (the
  padding rows are never written: a guard frame after the batch keeps its sentinel);
- spp != 1 has no direct form; invalid ranks are rejected before any work;
- FramePipeline(sub_bands=2): every group's frames equal single renders (animation cameras),
  counters too; sub_bands needs a slot count it divides;
- the gathered form of the groups (world > 1: one gather per group pass, un-permuted over
  W*S virtual ranks), run on one rank through a forced gather.
"""
import numpy as np
import pytest
import torch

from rust_tracer_amd import DeviceScene, RtError, SceneDesc, abi

pytestmark = pytest.mark.gpu


def cams_for(w, h, n, dx=0.05):
    out = []
    for k in range(n):
        c = abi.camera(w, h)
        c.origin[0] = c.origin[0] + dx * k
        out.append(c)
    return out


@pytest.mark.parametrize("w,h,world,n", [(200, 117, 2, 5), (160, 90, 3, 4), (96, 40, 4, 1)])
def test_direct_shares_fill_whole_frames(w, h, world, n):
    desc = SceneDesc.synth_config(3)
    s = DeviceScene(desc)
    shares = [s] + [s.clone(0) for _ in range(world - 1)]
    cams = cams_for(w, h, n)
    refs = [s.render(w, h, 8, cam=c, want_u8=True) for c in cams]
    frames = torch.full((n + 1, h, w, 3), float("nan"), dtype=torch.float32, device="cuda")
    frames8 = torch.full((n + 1, h, w, 3), 7, dtype=torch.uint8, device="cuda")
    cnt = [torch.zeros(3, dtype=torch.int64, device="cuda") for _ in range(world)]
    streams = [torch.cuda.Stream(torch.device("cuda", 0)) for _ in range(world)]
    main = torch.cuda.current_stream(0)
    for r in range(world):
        streams[r].wait_stream(main)
        with torch.cuda.stream(streams[r]):
            shares[r].render_bands_direct_async(cams, 8, 8, r, world, frames.data_ptr(), frames8.data_ptr(),
                                                cnt[r].data_ptr(), streams[r].cuda_stream)
    for st in streams:
        main.wait_stream(st)
    torch.cuda.synchronize()
    for sc in shares:
        sc.sync_status()
    got = frames.cpu().numpy()
    got8 = frames8.cpu().numpy()
    tot = [0, 0, 0]
    for k, (ref, c, _, ref8) in enumerate(refs):
        assert np.array_equal(got[k].view(np.uint32), ref.view(np.uint32)), f"frame {k}"
        assert np.array_equal(got8[k], ref8), f"frame {k} rgb8"
        tot = [tot[0] + c["node_rays"], tot[1] + c["shadow_rays"], tot[2] + c["pixels"]]
    assert np.isnan(got[n]).all() and (got8[n] == 7).all()  # nothing past the batch
    assert sum(x.cpu() for x in cnt).tolist() == tot
    for sc in shares[1:]:
        sc.close()
    s.close()


def test_direct_rejects_bad_arguments():
    s = DeviceScene(SceneDesc.synth_config(2))
    w, h = 64, 32
    buf = torch.zeros((1, h, w, 3), dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    with pytest.raises(RtError):
        s.render_bands_direct_async(cams_for(w, h, 1), 4, 8, 2, 2, buf.data_ptr(), 0, 0, st)
    with pytest.raises(RtError):
        s.render_bands_direct_async(cams_for(w, h, 1), 4, 8, 0, 2, 0, 0, 0, st)
    s.close()


def test_pipeline_sub_bands_equals_single_renders():
    from rust_tracer_amd.dist import FramePipeline
    desc = SceneDesc.synth_config(3)
    w, h, depth = 192, 108, 8
    s = DeviceScene(desc)
    pipe = FramePipeline(s, desc, w, h, depth, inflight=4, batch=3, sub_bands=2)
    assert pipe.groups == 2 and pipe.round_frames == 6

    def cam(i):
        c = abi.camera(w, h)
        c.origin[0] = 0.01 * (i % 64)
        return c
    lat = []
    pipe.run(8, lat, cameras=cam)  # passes of 3, 3, 2 frames on groups 0, 1, 0
    torch.cuda.synchronize()
    assert len(lat) == 6
    frames = pipe.frames()
    fc = pipe.frame_cameras()
    assert len(frames) == 5  # group 0's last pass (2 frames) + group 1's (3)
    tot = [0, 0, 0]
    for f, c in zip(frames, fc):
        ref, cnt, _, _ = s.render(w, h, depth, cam=c)
        assert np.array_equal(f.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    for i in range(8):
        _, cnt, _, _ = s.render(w, h, depth, cam=cam(i))
        tot = [tot[0] + cnt["node_rays"], tot[1] + cnt["shadow_rays"], tot[2] + cnt["pixels"]]
    assert pipe.counters.cpu().tolist() == tot
    whole = pipe.whole_tiler()
    one = whole.step()
    torch.cuda.synchronize()
    ref, _, _, _ = s.render(w, h, depth)
    assert np.array_equal(one.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    pipe.close()
    with pytest.raises(ValueError):
        FramePipeline(s, desc, w, h, depth, inflight=3, batch=2, sub_bands=2)
    s.close()


def test_pipeline_sub_bands_gathered_groups():
    """World > 1's form of the groups, on one rank: force_gather routes every group pass through
    one process-group gather (gloo, one rank) and the un-permute over W*S virtual ranks."""
    import os
    import socket

    import torch.distributed as dist
    from rust_tracer_amd.dist import FramePipeline
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        desc = SceneDesc.synth_config(3)
        w, h, depth = 160, 90, 8
        s = DeviceScene(desc)
        pipe = FramePipeline(s, desc, w, h, depth, inflight=4, batch=3, sub_bands=4, force_gather=True)
        assert pipe.group_gather and pipe.groups == 1

        def cam(i):
            c = abi.camera(w, h)
            c.origin[0] = 0.01 * (i % 64)
            return c
        pipe.run(6, cameras=cam)  # two passes of 3 frames on the one group
        torch.cuda.synchronize()
        frames, fc = pipe.frames(), pipe.frame_cameras()
        assert len(frames) == 3
        for f, c in zip(frames, fc):
            ref, _, _, _ = s.render(w, h, depth, cam=c)
            assert np.array_equal(f.cpu().numpy().view(np.uint32), ref.view(np.uint32))
        pipe.close()
        s.close()
    finally:
        dist.destroy_process_group()
