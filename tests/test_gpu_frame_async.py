"""GPU tests of rt_render_frame_async, the stream-ordered form of the drop-in seam
(render.rs:31-38 into device memory): rt_render's two band shares side by side on one device,
forked from and joined into the caller's stream.

- every frame equals rt_render bit for bit (f32, RGB8 and counters), over a run of calls
  whose meeting row moves with the shares' finish times, on config 3 at 1080p and at ragged
  sizes; frames under 32 rows take the one-pass path (padded and unpadded row counts);
- back-to-back calls without a host wait in between (the host never blocks) stay identical;
- a queue overflow in either share is reported by rt_scene_sync_status, never returned as a
  silent RT_OK, and the grown pools then render the full frame;
- a material edit reaches both shares' scene clones.
"""
import numpy as np
import pytest
import torch

from rust_tracer_amd import DeviceScene, RtError, SceneDesc, abi, phong_material

from .test_gpu_parity import _custom_scene

pytestmark = pytest.mark.gpu


def same_bits(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


class Dev:
    """Device buffers for one frame and the torch stream the renders are enqueued on."""

    def __init__(self, w, h):
        self.w, self.h = w, h
        self.rgb = torch.empty((h, w, 3), dtype=torch.float32, device="cuda:0")
        self.rgb8 = torch.empty((h, w, 3), dtype=torch.uint8, device="cuda:0")
        self.cnt = torch.zeros(3, dtype=torch.int64, device="cuda:0")
        self.side = torch.cuda.Stream(torch.device("cuda", 0))  # a created stream (rt_api.h)
        self.stream = self.side.cuda_stream

    def render(self, s, depth, cam=None, sync=True, want8=True):
        self.rgb.fill_(float("nan"))
        self.rgb8.fill_(7)
        self.cnt.zero_()
        self.side.wait_stream(torch.cuda.current_stream(0))  # the fills above come first
        cam = cam if cam is not None else abi.camera(self.w, self.h)
        s.render_frame_async(cam, depth, self.rgb.data_ptr(), self.cnt.data_ptr(), self.stream,
                             d_rgb8_ptr=self.rgb8.data_ptr() if want8 else 0)
        if sync:
            torch.cuda.synchronize()
            return self.host()

    def host(self):
        c = self.cnt.cpu().tolist()
        return (self.rgb.cpu().numpy(), self.rgb8.cpu().numpy(),
                {"node_rays": c[0], "shadow_rays": c[1], "pixels": c[2]})


@pytest.mark.parametrize("w,h", [(1920, 1080), (640, 361), (320, 20), (320, 24)])
def test_frame_async_equals_render(w, h):
    desc = SceneDesc.synth_config(3)
    s = DeviceScene(desc, device=0)
    ref, rcnt, _, ref8 = s.render(w, h, 8, want_u8=True)
    d = Dev(w, h)
    for i in range(8):  # synchronised calls: the meeting row may move between them
        img, img8, cnt = d.render(s, 8)
        assert same_bits(img, ref), f"call {i}: frame differs"
        assert np.array_equal(img8, ref8), f"call {i}: RGB8 differs"
        assert cnt == rcnt, (i, cnt, rcnt)
    s.sync_status()
    s.close()


def test_frame_async_back_to_back_and_cameras():
    """Calls enqueued without a host wait (each its own camera, its own output buffers) equal
    rt_render of that camera."""
    desc = SceneDesc.synth_config(3)
    w, h = 640, 360
    s = DeviceScene(desc, device=0)
    cams = []
    for i in range(4):
        c = abi.camera(w, h)
        c.origin[0] = 0.05 * i
        cams.append(c)
    refs = [s.render(w, h, 8, cam=c)[0] for c in cams]
    devs = [Dev(w, h) for _ in cams]
    for d, c in zip(devs, cams):
        d.render(s, 8, cam=c, sync=False, want8=False)
    torch.cuda.synchronize()
    s.sync_status()
    for i, (d, ref) in enumerate(zip(devs, refs)):
        assert same_bits(d.rgb.cpu().numpy(), ref), f"frame {i} differs"
    s.close()


def test_frame_async_overflow_is_reported(monkeypatch):
    """Pools far too small: the call returns (stream-ordered), rt_scene_sync_status raises
    RT_ERR_CAPACITY; renders after it grow the pools until the full frame fits."""
    desc = SceneDesc.synth_config(3)
    w, h = 256, 144
    full = DeviceScene(desc, device=0)
    ref, rcnt, _, _ = full.render(w, h, 8)
    full.close()
    s = DeviceScene(desc, device=0, tuning=f"node_cap={w * h // 2 + 4096}")
    d = Dev(w, h)
    d.render(s, 8, want8=False)
    with pytest.raises(RtError) as e:
        s.sync_status()
    assert e.value.status == abi.RT_ERR_CAPACITY
    s.sync_status()  # cleared once reported
    # an rt_render between the call and the status check (same band shares) does not swallow
    # the report
    d.render(s, 8, want8=False)
    img_r, cnt_r, _, _ = s.render(w, h, 8)
    assert same_bits(img_r, ref) and cnt_r == rcnt
    with pytest.raises(RtError) as e:
        s.sync_status()
    assert e.value.status == abi.RT_ERR_CAPACITY
    for _ in range(12):
        img, _, cnt = d.render(s, 8, want8=False)
        try:
            s.sync_status()
        except RtError as err:
            assert err.status == abi.RT_ERR_CAPACITY
            continue
        break
    else:
        pytest.fail("the pools never grew enough")
    assert same_bits(img, ref) and cnt == rcnt
    s.close()


def test_frame_async_after_material_edit():
    desc = _custom_scene()
    w, h = 320, 240
    s = DeviceScene(desc, device=0)
    d = Dev(w, h)
    d.render(s, 8)
    m = phong_material((0.05, 0.0, 0.0), (0.2, 0.9, 0.3), (0.5, 0.5, 0.5), 30.0, 0.0, 0.0)
    s.set_material(3, m)
    img, img8, cnt = d.render(s, 8)
    ref, rcnt, _, ref8 = s.render(w, h, 8, want_u8=True)
    assert same_bits(img, ref) and np.array_equal(img8, ref8) and cnt == rcnt
    s.close()
