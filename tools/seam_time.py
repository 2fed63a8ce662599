"""Times the single-frame seam (render.rs:31's render() through the C ABI) on config 3:
one pass on one stream (device-resident), rt_render with its pageable / page-locked host
copy, and rt_render on a scene tiled over S band shares of the same GPU (devices = [0] * S:
S passes on S streams, device copies, un-permute).  Prints one JSON line.
usage: python tools/seam_time.py [S ...]   (env RT_* switches apply)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rust_tracer_amd import DeviceScene, HostFrame, SceneDesc, abi  # noqa: E402


def best(f, n=5):
    f()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append((time.perf_counter() - t0) * 1e3)
    return round(min(ts), 3)


def main():
    w, h, depth = 1920, 1080, 8
    desc = SceneDesc.synth_config(3)
    s = DeviceScene(desc, device=0)
    out = {"env": {k: v for k, v in os.environ.items() if k.startswith("RT_")}}
    dev = torch.device("cuda", 0)
    band = torch.zeros((1088, w, 3), device=dev)
    cnt = torch.zeros(3, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev)
    cam = abi.camera(w, h)

    def one():
        s.render_bands_async(cam, depth, 8, 0, 1, band.data_ptr(), cnt.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
    one()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(10):
        s.render_bands_async(cam, depth, 8, 0, 1, band.data_ptr(), cnt.data_ptr(), st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    out["one_pass_ms"] = round(e0.elapsed_time(e1) / 10, 4)
    ref = band[:h].cpu().numpy()
    out["rt_render_pageable_ms"] = best(lambda: s.render(w, h, depth))
    out["rt_render_device_ms"] = round(min(s.render(w, h, depth)[2] for _ in range(5)), 4)
    hf = HostFrame(w, h)
    out["rt_render_pinned_ms"] = best(lambda: s.render(w, h, depth, out=hf.array))
    img = s.render(w, h, depth, out=hf.array)[0]
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
    s.close()
    for S in [int(a) for a in sys.argv[1:]]:
        m = DeviceScene(desc, devices=[0] * S)
        out[f"split{S}_pinned_ms"] = best(lambda: m.render(w, h, depth, out=hf.array))
        img = m.render(w, h, depth, out=hf.array)
        out[f"split{S}_kernel_ms"] = round(img[2], 4)
        assert np.array_equal(img[0].view(np.uint32), ref.view(np.uint32))
        m.close()
    hf.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
