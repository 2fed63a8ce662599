"""A/B of render-pipeline switches (RT_* environment variables) at bench.py's default
throughput regime: F frames in flight (F scene handles, one HIP stream each).

usage: python tools/ab_inflight.py [config=3] [frames=24] VAR=VAL[,VAR=VAL...] ...
Each argument after the first two is one variant ("-" = defaults); env FLIGHT (default 4),
REPS (default 3).  Prints the median ms per frame (wall clock over `frames` frames) and
checks every variant's frame is bit-identical to the first variant's.
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rust_tracer_amd import DeviceScene, SceneDesc, abi  # noqa: E402


def main():
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    variants = sys.argv[3:] or ["-"]
    flight = int(os.environ.get("FLIGHT", "4"))
    reps = int(os.environ.get("REPS", "3"))
    depth = 4 if config == 2 else 8
    w, h = 1920, 1080
    cam = abi.camera(w, h)
    desc = SceneDesc.synth_config(config)
    streams = [torch.cuda.Stream() for _ in range(flight)]
    bufs = [torch.zeros((h, w, 3), dtype=torch.float32, device="cuda") for _ in range(flight)]
    cnts = [torch.zeros(3, dtype=torch.int64, device="cuda") for _ in range(flight)]
    ref = None
    for v in variants:
        env = {} if v == "-" else dict(kv.split("=", 1) for kv in v.split(","))
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            scenes = [DeviceScene(desc) for _ in range(flight)]
            times = []
            for rep in range(reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k in range(frames):
                    i = k % flight
                    scenes[i].render_bands_async(cam, depth, 8, 0, 1, bufs[i].data_ptr(), cnts[i].data_ptr(),
                                                 streams[i].cuda_stream)
                torch.cuda.synchronize()
                if rep:
                    times.append((time.perf_counter() - t0) / frames * 1e3)
            for s in scenes:
                s.close()
        finally:
            for k, val in old.items():
                if val is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = val
        img = bufs[0].cpu().numpy()
        same = None
        if ref is None:
            ref = img
        else:
            same = bool(np.array_equal(ref.view(np.uint32), img.view(np.uint32)))
        print(f"{v:40s} median {np.median(times):8.3f} ms/frame  min {min(times):8.3f}  identical={same}",
              flush=True)


if __name__ == "__main__":
    main()
