"""Timing of rt_render_frame_async (the stream-ordered seam split) against one pipeline pass
and rt_render, config 3 at 1080p; optionally after building a FramePipeline (more streams).
usage: python tools/frame_async_time.py [--pipeline 0|1] [--n 5]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tracer_amd import DeviceScene, SceneDesc, abi  # noqa: E402
from rust_tracer_amd.dist import FramePipeline, FrameTiler  # noqa: E402


def timed(fn, n, sync_each):
    main = torch.cuda.current_stream(0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    for _ in range(n):
        fn()
        if sync_each:
            torch.cuda.synchronize()
    e1.record(main)
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pipeline", type=int, default=0)
    ap.add_argument("--n", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--render-first", type=int, default=0, help="rt_render calls before the split tiler")
    ap.add_argument("--pinned", type=int, default=0, help="those rt_render calls into page-locked memory")
    ap.add_argument("--stream", default="default", help="default | side (a torch side stream)")
    a = ap.parse_args()
    w, h, depth = 1920, 1080, 8
    desc = SceneDesc.synth_config(3)
    s = DeviceScene(desc, device=0)
    dev = torch.device("cuda", 0)
    out = {"env_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}
    if a.pipeline:
        pipe = FramePipeline(s, desc, w, h, depth, 8, 0, 1, dev, inflight=4, batch=a.batch)
        pipe.run(4 * a.batch)
        torch.cuda.synchronize()
        s.set_grid_share(100)
    hf = None
    if a.pinned:
        from rust_tracer_amd import HostFrame
        hf = HostFrame(w, h)
    for _ in range(a.render_first):
        s.render(w, h, depth, out=hf.array if hf is not None else None)
    side = torch.cuda.Stream(dev) if a.stream == "side" else None
    ctx = torch.cuda.stream(side) if side is not None else torch.cuda.stream(torch.cuda.current_stream(dev))
    with ctx:
        one = FrameTiler(s, w, h, depth, device=dev)
        sp = FrameTiler(s, w, h, depth, device=dev, split=True)
        for t in (one, sp):
            for _ in range(3):
                t.step()
                torch.cuda.synchronize()
        out["one_pass_ms"] = timed(one.step, a.n, False)
        out["split_back_to_back_ms"] = timed(sp.step, a.n, False)
        out["split_synced_ms"] = timed(sp.step, a.n, True)
        out["one_pass_synced_ms"] = timed(one.step, a.n, True)
    s.sync_status()
    out["identical"] = bool(torch.equal(one.frame, sp.frame))
    ms = []
    for _ in range(a.n):
        _, _, k, _ = s.render(w, h, depth)
        ms.append(k)
    out["rt_render_device_ms"] = round(min(ms), 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
