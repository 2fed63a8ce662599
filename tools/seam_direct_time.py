"""One frame at a time through S band shares of one device writing in place
(rt_render_bands_direct_async: S scene handles on S streams forked from and joined into one
stream, 8-row bands dealt over the shares) against rt_render_frame_async (two contiguous
shares), config 3 at 1080p.  Device time per frame over back-to-back frames.
usage: python tools/seam_direct_time.py [n=10]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tracer_amd import DeviceScene, SceneDesc, abi  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10
W, H, DEPTH = 1920, 1080, 8
dev = torch.device("cuda", 0)
scene = DeviceScene(SceneDesc.synth_config(3))
clones = [scene.clone(0) for _ in range(5)]
side = torch.cuda.Stream(dev)
streams = [torch.cuda.Stream(dev) for _ in range(6)]
frame = torch.zeros((1, H, W, 3), dtype=torch.float32, device=dev)
cnt = torch.zeros(3, dtype=torch.int64, device=dev)
cam = [abi.camera(W, H)]
ref, _, _, _ = scene.render(W, H, DEPTH)


def direct(S, band):
    shares = ([scene] + clones)[:S]
    for j, sc in enumerate(shares):
        streams[j].wait_stream(side)
        with torch.cuda.stream(streams[j]):
            sc.render_bands_direct_async(cam, DEPTH, band, j, S, frame.data_ptr(), 0, cnt.data_ptr(),
                                         streams[j].cuda_stream)
        side.wait_stream(streams[j])


def split():
    scene.render_frame_async(cam[0], DEPTH, frame.data_ptr(), cnt.data_ptr(), side.cuda_stream)


def timed(fn):
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(side)
        for _ in range(N):
            fn()
        e1.record(side)
    torch.cuda.synchronize()
    same = bool(torch.equal(frame[0].cpu().view(torch.int32), torch.from_numpy(ref).view(torch.int32)))
    return round(e0.elapsed_time(e1) / N, 4), same


out = {"split": timed(split)}
for pct in (100, 80, 60):
    for sc in [scene] + clones:
        sc.set_grid_share(pct)
    for S in (1, 2, 3, 4):
        for band in (8, 32):
            if S == 1 and band == 32:
                continue
            out[f"S{S}_band{band}_grid{pct}"] = timed(lambda: direct(S, band))
for sc in [scene] + clones:
    sc.sync_status()
print(json.dumps(out, indent=0))
